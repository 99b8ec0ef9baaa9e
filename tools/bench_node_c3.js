'use strict';
// BASELINE config 3 through the Node drop-in host: `splat-transform in.ply -r 0,45,0 --filterNaN
// out.compressed.ply` as the reference's index.ts:101-154 + 463-496 drive it, i.e.
// compressPlyFile(inHandle, outHandle, actions) of splat-transform_amd/js over the N-API addon
// (readPly + processDataTable + writeCompressedPly, the arrays written into the file as they
// leave HBM).  Every rep writes a fresh output ('wx', as the reference's CLI).
//   node tools/bench_node_c3.js <in.ply> <dir> <reps>
// Rep 0 warms; reps 1.. are timed.  Prints one JSON line: per-rep ms and each output's sha256.
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', 'splat-transform_amd', 'js'));

(async () => {
    const [src, dir] = process.argv.slice(2, 4);
    const reps = parseInt(process.argv[4] || '3', 10);
    const actions = [{ kind: 'rotate', value: { x: 0, y: 45, z: 0 } }, { kind: 'filterNaN' }];
    const ms = [];
    const split = [];
    const sha = [];
    const d = (a, b) => Number(b - a) / 1e6;
    for (let r = 0; r <= reps; ++r) {
        const dst = path.join(dir, `node${r}.compressed.ply`);
        const t0 = process.hrtime.bigint();
        const inH = await fs.promises.open(src, 'r');
        const outH = await fs.promises.open(dst, 'wx');
        const t1 = process.hrtime.bigint();
        await host.compressPlyFile(inH, outH, actions);
        const t2 = process.hrtime.bigint();
        await outH.close();
        await inH.close();
        const t3 = process.hrtime.bigint();
        if (r) {
            ms.push(d(t0, t3));
            split.push({ open: d(t0, t1), call: d(t1, t2), close: d(t2, t3) });
        }
        sha.push(crypto.createHash('sha256').update(fs.readFileSync(dst)).digest('hex'));
        fs.unlinkSync(dst);
    }
    console.log(JSON.stringify({ ms, split, sha256: sha }));
})().catch((e) => { console.error(e); process.exit(1); });
