'use strict';
// writeSogFile (the archive streamed into an open file) or writeSogBundle on a table, seeded
// Math.random stream and pinned clock; the test compares the two outputs.
//   node sog_file.js <dir> file|bundle      (dir holds manifest.json + <col>.f32)
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
const mode = process.argv[3] || 'file';
const man = JSON.parse(fs.readFileSync(path.join(dir, 'manifest.json'), 'utf8'));
const readF32 = (name) => {
    const b = fs.readFileSync(path.join(dir, name + '.f32'));
    return new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength));
};
const dt = new host.DataTable(man.columns.map(n => new host.Column(n, readF32(n))));
const RealDate = Date;
global.Date = class extends RealDate { constructor(...a) { super(...(a.length ? a : man.clock)); } };
(async () => {
    // one writer per process: the host's draw pool keeps what a call did not use
    Math.random = mulberry32(man.seed);
    if (mode === 'bundle') {
        fs.writeFileSync(path.join(dir, 'out_bundle.sog'), await host.writeSogBundle(dt, man.iters));
    } else {
        const fh = await fs.promises.open(path.join(dir, 'out_file.sog'), 'w');
        const size = await host.writeSogFile(fh, dt, man.iters);
        await fh.close();
        if (size !== fs.statSync(path.join(dir, 'out_file.sog')).size) {
            console.error('size mismatch', size);
            process.exit(1);
        }
    }
    global.Date = RealDate;
    console.log('sog ' + mode + ' ok');
})().catch((e) => { console.error(e); process.exit(1); });
