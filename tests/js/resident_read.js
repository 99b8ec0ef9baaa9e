'use strict';
// readPly's resident columns (the addon's st_ply_read_resident: the values stay in HBM until JS
// reads a column's `data`) through writeSogFile.  Every write starts Math.random on the same
// stream and Date on a pinned clock, so equal tables must give equal archives:
//   untouched      no column read by JS: every writeSog column taken from HBM
//   read           JS read every column (copied down): all of them uploaded
//   changed        one value of f_rest_3 changed: that column uploaded, the other 58 from HBM
//   changed_ref    the same change after reading every column: all uploaded
//   first, second  two reads of the file, both tables alive: each keeps its own device copy
//   bundle         writeSogBundle of an untouched table (st_sog_bundle): the same bytes, from HBM
//   meta           numRows / names / getColumnByName only: still from HBM
// Prints one JSON line {case: {sha, reused}, ..., numRows}.
//   node resident_read.js <in.ply> <dir> <iters>
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', '..', 'splat-transform_amd', 'js'));

const [src, dir, itersArg] = process.argv.slice(2);
const iters = parseInt(itersArg || '3', 10);
const RealDate = Date;
global.Date = class extends RealDate { constructor(...a) { super(...(a.length ? a : [2024, 0, 1, 0, 0, 0])); } };

const fixDraws = () => {
    let s = 12345;
    Math.random = () => {
        s = (s * 16807) % 2147483647;
        return (s - 1) / 2147483646;
    };
    host.resetRandomStream();
};

const read = async () => {
    const fh = await fs.promises.open(src, 'r');
    const ply = await host.readPly(fh);
    await fh.close();
    return ply.elements.find(e => e.name === 'vertex').dataTable;
};

const write = async (table, name) => {
    fixDraws();
    const out = path.join(dir, name);
    const fh = await fs.promises.open(out, 'w');
    await host.writeSogFile(fh, table, iters);
    await fh.close();
    const sha = crypto.createHash('sha256').update(fs.readFileSync(out)).digest('hex');
    return { sha, reused: host.addon.lastHostReuse().columns };
};

(async () => {
    const res = {};
    res.untouched = await write(await read(), 'a.sog');

    let t = await read();
    let sum = 0;
    for (const c of t.columns) sum += c.data[0];
    res.read = await write(t, 'b.sog');
    res.read.finite = Number.isFinite(sum);

    t = await read();
    const col = t.getColumnByName('f_rest_3');
    col.data[7] = col.data[7] + 0.5;
    res.changed = await write(t, 'c.sog');

    t = await read();
    for (const c of t.columns) sum += c.data.length;
    const col2 = t.getColumnByName('f_rest_3');
    col2.data[7] = col2.data[7] + 0.5;
    res.changed_ref = await write(t, 'd.sog');

    const t1 = await read();
    const t2 = await read();
    res.first = await write(t1, 'e.sog');
    res.second = await write(t2, 'f.sog');

    // writeSogBundle of an untouched table: the same archive from HBM
    t = await read();
    fixDraws();
    const bundle = await host.writeSogBundle(t, iters);
    res.bundle = { sha: crypto.createHash('sha256').update(bundle).digest('hex'), reused: host.addon.lastHostReuse().columns };

    t = await read();
    res.numRows = t.numRows;
    res.columns = t.columns.map(c => c.name).length;
    res.hasRot = t.hasColumn('rot_0') && !!t.getColumnByName('rot_0');
    res.meta = await write(t, 'g.sog');
    // the first table's values (copied down here, after the second read), as bytes
    fs.writeFileSync(path.join(dir, 'first_f_rest_44.bin'), Buffer.from(t1.getColumnByName('f_rest_44').data.buffer));
    fs.writeFileSync(path.join(dir, 'meta_x.bin'), Buffer.from(t.getColumnByName('x').data.buffer));
    console.log(JSON.stringify(res));
})().catch((e) => { console.error(e); process.exit(1); });
