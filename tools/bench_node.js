'use strict';
// The reference CLI's job for `splat-transform in.ply out.sog` through the Node drop-in host
// (splat-transform_amd/js: readPly -> writeSogFile over the N-API addon), the way the reference's
// index.ts:433-510 drives it: the PLY is read into a host DataTable (readers/read-ply.ts:111-191),
// then writeSog writes the .sog into an open FileHandle (writers/write-sog.ts:110-370).
//   node tools/bench_node.js <in.ply> <out.sog> <reps> <iters> [<draws.f64> <clock json>]
// Rep 0 warms the addon, the device buffers and the page cache; reps 1.. are timed.  Prints one
// JSON line: per-rep milliseconds of readPly, writeSogFile and the whole job, the .sog size and
// each rep's sha256 of the file.  With a draws file (little-endian f64) every rep starts
// Math.random on that stream and Date on the given clock ([y, m, d, h, min, s]), so the archive
// is fixed: bench.py checks it against the library's own archive of the same step.
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', 'splat-transform_amd', 'js'));

const ms = (a, b) => Number(b - a) / 1e6;

(async () => {
    const [src, dst] = process.argv.slice(2, 4);
    const reps = parseInt(process.argv[4] || '2', 10);
    const iters = parseInt(process.argv[5] || '10', 10);
    const drawsFile = process.argv[6];
    const clock = process.argv[7] ? JSON.parse(process.argv[7]) : null;
    let draws = null;
    if (drawsFile) {
        const b = fs.readFileSync(drawsFile);
        draws = new Float64Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength));
    }
    if (clock) {
        const RealDate = Date;
        global.Date = class extends RealDate { constructor(...a) { super(...(a.length ? a : clock)); } };
    }
    const runs = [];
    const sha = [];
    let size = 0;
    let rows = 0;
    for (let r = 0; r <= reps; ++r) {
        // the last rep's table is garbage: collected here (node --expose-gc), outside the timed
        // region, its column blocks go back to the addon's pool -- every timed readPly writes
        // into faulted-in pages, as in the rep after a collection (a CLI process reads once, into
        // fresh pages: ~+40 ms at 10M splats)
        if (typeof global.gc === 'function') global.gc();
        if (draws) {  // the same stream for every rep (outside the timed region)
            let i = 0;
            Math.random = () => {
                if (i >= draws.length) throw new Error('bench_node: the draws file ran out');
                return draws[i++];
            };
            host.resetRandomStream();
        }
        const t0 = process.hrtime.bigint();
        const inH = await fs.promises.open(src, 'r');
        const ply = await host.readPly(inH);
        await inH.close();
        const t1 = process.hrtime.bigint();
        const table = ply.elements.find(e => e.name === 'vertex').dataTable;
        rows = table.numRows;
        // no O_TRUNC: writeSogFile cuts the file to the archive's length (a file truncated to zero and
        // rewritten is flushed at close on ext4, and frees its old pages first)
        const outH = await fs.promises.open(dst, fs.constants.O_WRONLY | fs.constants.O_CREAT, 0o644);
        const t1b = process.hrtime.bigint();
        size = await host.writeSogFile(outH, table, iters);
        const t1c = process.hrtime.bigint();
        await outH.close();
        const t2 = process.hrtime.bigint();
        if (r) {
            runs.push({ readPly: ms(t0, t1), writeSogFile: ms(t1, t2), total: ms(t0, t2),
                open: ms(t1, t1b), write: ms(t1b, t1c), close: ms(t1c, t2),
                reusedColumns: host.addon.lastHostReuse().columns });
        }
        sha.push(crypto.createHash('sha256').update(fs.readFileSync(dst)).digest('hex'));
    }
    if (size !== fs.statSync(dst).size) throw new Error('writeSogFile size mismatch');
    console.log(JSON.stringify({ rows, sog_bytes: size, runs, sha256: sha }));
})().catch((e) => { console.error(e); process.exit(1); });
