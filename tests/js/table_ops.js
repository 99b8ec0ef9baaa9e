'use strict';
// Node host: filterNaN / combine / transform's column-type rule on the reference's own vectors
// (tests/golden/filter_combine.*).  Prints one JSON object of check results.
//   node table_ops.js combine|filter|devices
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', '..', 'splat-transform_amd', 'js'));
const GOLDEN = path.join(__dirname, '..', 'golden');

const CTOR = { f4: Float32Array, f8: Float64Array, u4: Uint32Array, i4: Int32Array, u1: Uint8Array, i1: Int8Array,
    u2: Uint16Array, i2: Int16Array };
const man = JSON.parse(fs.readFileSync(path.join(GOLDEN, 'filter_combine.json'), 'utf8'));
const blob = fs.readFileSync(path.join(GOLDEN, 'filter_combine.bin'));
const arr = (k) => {
    const a = man.arrays[k];
    const ctor = CTOR[a.dtype];
    const copy = Buffer.from(blob.subarray(a.offset, a.offset + a.nbytes));
    return new ctor(copy.buffer, copy.byteOffset, a.nbytes / ctor.BYTES_PER_ELEMENT);
};
const sameBytes = (a, b) => a.constructor === b.constructor && a.length === b.length &&
    Buffer.from(a.buffer, a.byteOffset, a.byteLength).equals(Buffer.from(b.buffer, b.byteOffset, b.byteLength));

const out = {};
const what = process.argv[2];
if (what === 'combine') {
    const tables = [0, 1, 2, 3].map(i => new host.DataTable(man.meta[`c4_${i}_names`].map((n, j) =>
        new host.Column(n, arr(`c4_${i}_i${j}`)))));
    const merged = host.combine(tables);
    out.names = merged.columns.map(c => c.name);
    out.same = merged.columns.map((c, j) => sameBytes(c.data, arr(`c4_out_i${j}`)));
    const abc = ['a', 'b', 'c'].map(t => new host.DataTable(man.meta[`cmb_${t}_columns`].map(n =>
        new host.Column(n, arr(`cmb_${t}_${n}`)))));
    const m3 = host.combine(abc);
    out.same3 = m3.columns.map((c, j) => sameBytes(c.data, arr(`cmb_out_i${j}`)));
} else if (what === 'filter') {
    const table = new host.DataTable(man.meta.typed_in_columns.map(n => new host.Column(n, arr(`typed_in_${n}`))));
    const res = host.filterNaN(table);
    out.same = res.columns.map(c => sameBytes(c.data, arr(`typed_out_${c.name}`)));
    const splats = new host.DataTable(man.meta.in_columns.map(n => new host.Column(n, arr(`in_${n}`))));
    const res2 = host.filterNaN(splats);
    out.same2 = res2.columns.map(c => sameBytes(c.data, arr(`out_${c.name}`)));
} else if (what === 'devices') {
    out.before = host.getDevices();
    host.setDevices(1);
    out.after = host.getDevices();
    try {
        host.setDevices(1000);
        out.threw = false;
    } catch (e) {
        out.threw = /status -1\)/.test(e.message);
    }
}
console.log(JSON.stringify(out));
