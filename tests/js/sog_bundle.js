'use strict';
// writeSog to a .sog through the Node host module (writeSogBundle, WebpEncoder), on a
// table written by tests/test_js_host.py; Math.random is the fixture's seeded stream and
// Date the fixture's pinned clock (tests/golden/gen/make_golden.js, case sog_bundle).
//   node sog_bundle.js <dir>      (dir holds manifest.json + <col>.f32 + img.rgba)
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
Math.random = mulberry32(man.seed);
const RealDate = Date;
global.Date = class extends RealDate { constructor(...a) { super(...(a.length ? a : man.clock)); } };
host.writeSogBundle(dt, man.iters).then(async (archive) => {
    global.Date = RealDate;
    fs.writeFileSync(path.join(dir, 'out.sog'), archive);
    const img = fs.readFileSync(path.join(dir, 'img.rgba'));
    const enc = await host.WebpEncoder.create();
    fs.writeFileSync(path.join(dir, 'img.webp'), enc.encodeLosslessRGBA(new Uint8Array(img), man.w, man.h));
    console.log('sog bundle ok');
}).catch((e) => { console.error(e); process.exit(1); });
