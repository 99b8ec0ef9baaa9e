'use strict';
// readPly / isCompressedPly / decompressPly through the Node host module on files written by
// tests/test_js_host.py; every column is dumped as raw bytes for the comparison.
//   node ply_read.js <dir>      (dir holds mixed.ply and comp.ply)
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', '..', 'splat-transform_amd', 'js'));

const dir = process.argv[2];
const dump = (name, ta) => fs.writeFileSync(path.join(dir, name), Buffer.from(ta.buffer, ta.byteOffset, ta.byteLength));

(async () => {
    const summary = {};
    for (const f of ['mixed', 'comp']) {
        const fh = await fs.promises.open(path.join(dir, f + '.ply'), 'r');
        const ply = await host.readPly(fh);
        await fh.close();
        summary[f] = { comments: ply.comments, elements: ply.elements.map(e => [e.name, e.dataTable.numRows,
            e.dataTable.columns.map(c => [c.name, c.data.constructor.name])]), compressed: host.isCompressedPly(ply) };
        for (const e of ply.elements) for (const c of e.dataTable.columns) dump(`${f}_${e.name}_${c.name}.bin`, c.data);
        if (summary[f].compressed) {
            const dt = host.decompressPly(ply);
            summary[f].decoded = dt.columns.map(c => c.name);
            for (const c of dt.columns) dump(`${f}_dec_${c.name}.bin`, c.data);
        }
    }
    fs.writeFileSync(path.join(dir, 'summary.json'), JSON.stringify(summary));
    console.log('ply read ok');
})().catch((e) => { console.error(e); process.exit(1); });
