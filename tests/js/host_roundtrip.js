'use strict';
// Drives the Node host module (splat-transform_amd/js) the way the reference's
// writers call the hot path, on columns written by tests/test_js_host.py:
//   transform(-r 0,45,0) -> generateOrdering + chunk pack -> kmeans(f_rest, k, iters)
// Math.random is the seeded mulberry32 stream of tests/golden/gen/make_golden.js.
//   node host_roundtrip.js <dir>      (dir holds manifest.json + <col>.f32)
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', '..', 'splat-transform_amd', 'js'));

const mulberry32 = (seed) => {
    let a = seed >>> 0;
    return () => {
        a = (a + 0x6D2B79F5) >>> 0;
        let t = a;
        t = Math.imul(t ^ (t >>> 15), t | 1);
        t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
        return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
    };
};

const dir = process.argv[2];
const man = JSON.parse(fs.readFileSync(path.join(dir, 'manifest.json'), 'utf8'));
Math.random = mulberry32(man.seed);
const readF32 = (name) => {
    const b = fs.readFileSync(path.join(dir, name + '.f32'));
    return new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength));
};
const writeRaw = (name, ta) => fs.writeFileSync(path.join(dir, name), Buffer.from(ta.buffer, ta.byteOffset, ta.byteLength));

const dt = new host.DataTable(man.columns.map(n => new host.Column(n, readF32(n))));
const q = host.quatFromEuler(man.euler[0], man.euler[1], man.euler[2]);
host.transform(dt, { x: 0, y: 0, z: 0 }, q, 1);
for (const c of dt.columns) writeRaw('t_' + c.name + '.f32', c.data);

const packed = host.packCompressed(dt);
writeRaw('chunk.f32', packed.chunk);
writeRaw('vertex.u32', packed.vertex);
writeRaw('sh.u8', packed.sh);

const shCols = dt.columns.filter(c => c.name.startsWith('f_rest_'));
host.kmeans(new host.DataTable(shCols), man.k, man.iters).then((res) => {
    writeRaw('labels.u32', res.labels);
    const d = res.centroids.numColumns;
    const kk = res.centroids.numRows;
    const cen = new Float32Array(d * kk);
    for (let i = 0; i < d; ++i) cen.set(res.centroids.getColumn(i).data, i * kk);
    writeRaw('centroids.f32', cen);
    console.log('host roundtrip ok');
}).catch((e) => { console.error(e); process.exit(1); });
