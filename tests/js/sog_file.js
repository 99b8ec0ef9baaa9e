'use strict';
// writeSogFile (the archive streamed into an open file) against writeSogBundle on the same
// table, Math.random stream and clock: the file must hold the bundle's bytes.
//   node sog_file.js <dir>      (dir holds manifest.json + <col>.f32)
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
const readF32 = (name) => {
    const b = fs.readFileSync(path.join(dir, name + '.f32'));
    return new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength));
};
const dt = new host.DataTable(man.columns.map(n => new host.Column(n, readF32(n))));
const RealDate = Date;
global.Date = class extends RealDate { constructor(...a) { super(...(a.length ? a : man.clock)); } };
(async () => {
    Math.random = mulberry32(man.seed);
    const archive = await host.writeSogBundle(dt, man.iters);
    Math.random = mulberry32(man.seed);
    const fh = await fs.promises.open(path.join(dir, 'out_file.sog'), 'w');
    const size = await host.writeSogFile(fh, dt, man.iters);
    await fh.close();
    global.Date = RealDate;
    const got = fs.readFileSync(path.join(dir, 'out_file.sog'));
    if (size !== got.length || !got.equals(Buffer.from(archive))) {
        console.error('file differs from the bundle', size, got.length, archive.length);
        process.exit(1);
    }
    console.log('sog file ok', size);
})().catch((e) => { console.error(e); process.exit(1); });
