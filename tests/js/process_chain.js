'use strict';
// Node host: processDataTable and writeCompressedPly (with the actions in the same device call)
// on the reference's own vectors (tests/golden/process_chain.*).  Prints one JSON object:
// per case, whether the processed table and the four compressed-PLY writes match byte for byte.
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', '..', 'splat-transform_amd', 'js'));
const GOLDEN = path.join(__dirname, '..', 'golden');

const CTOR = { f4: Float32Array, f8: Float64Array, u4: Uint32Array, i4: Int32Array, u1: Uint8Array, i1: Int8Array,
    u2: Uint16Array, i2: Int16Array };
const man = JSON.parse(fs.readFileSync(path.join(GOLDEN, 'process_chain.json'), 'utf8'));
const blob = fs.readFileSync(path.join(GOLDEN, 'process_chain.bin'));
const arr = (k) => {
    const a = man.arrays[k];
    const ctor = CTOR[a.dtype];
    const copy = Buffer.from(blob.subarray(a.offset, a.offset + a.nbytes));
    return new ctor(copy.buffer, copy.byteOffset, a.nbytes / ctor.BYTES_PER_ELEMENT);
};
const bytes = a => Buffer.from(a.buffer, a.byteOffset, a.byteLength);
const sameBytes = (a, b) => a.constructor === b.constructor && a.length === b.length && bytes(a).equals(bytes(b));
// the fixture stores Vec3 action values as [x, y, z]
const actionsOf = c => man.meta[`${c}_actions`].map(a => (Array.isArray(a.value)
    ? Object.assign({}, a, { value: { x: a.value[0], y: a.value[1], z: a.value[2] } }) : a));
const tableOf = c => new host.DataTable(man.meta[`${c}_in_columns`].map(n => new host.Column(n, arr(`${c}_in_${n}`))));

(async () => {
    const out = {};
    for (const c of man.meta.cases) {
        const r = {};
        const input = tableOf(c);
        const res = host.processDataTable(input, actionsOf(c));
        // the caller's table afterwards (transforms before the first filter mutate it in place)
        r.after = input.columns.every(col => sameBytes(col.data, arr(`${c}_after_${col.name}`)));
        r.names = JSON.stringify(res.columns.map(col => col.name)) === JSON.stringify(man.meta[`${c}_out_columns`]);
        r.table = res.columns.every(col => sameBytes(col.data, arr(`${c}_out_${col.name}`)));
        const writes = [];
        const fh = { write: async (d) => { writes.push(Buffer.from(d.buffer, d.byteOffset, d.byteLength)); } };
        await host.writeCompressedPly(fh, tableOf(c), actionsOf(c));
        r.writes = writes.length === 4 && ['header', 'chunk', 'vertex', 'sh'].every((k, i) => writes[i].equals(bytes(arr(`${c}_${k}`))));
        // the reference's split: processDataTable, then writeCompressedPly of its result
        const w2 = [];
        await host.writeCompressedPly({ write: async (d) => { w2.push(Buffer.from(d.buffer, d.byteOffset, d.byteLength)); } }, res);
        r.writes2 = w2.length === 4 && ['header', 'chunk', 'vertex', 'sh'].every((k, i) => w2[i].equals(bytes(arr(`${c}_${k}`))));
        // the same from a PLY file of the input table (readPly + actions + writer in one call)
        const dir = fs.mkdtempSync(path.join(require('os').tmpdir(), 'st_chain_'));
        const names = man.meta[`${c}_in_columns`];
        const n = arr(`${c}_in_${names[0]}`).length;
        const header = Buffer.from(['ply', 'format binary_little_endian 1.0', `element vertex ${n}`]
            .concat(names.map(nm => `property float ${nm}`), 'end_header\n').join('\n'), 'utf8');
        const rows = Buffer.alloc(n * 4 * names.length);
        const cols = names.map(nm => arr(`${c}_in_${nm}`));
        for (let i = 0; i < n; ++i) for (let j = 0; j < names.length; ++j) rows.writeFloatLE(cols[j][i], (i * names.length + j) * 4);
        fs.writeFileSync(path.join(dir, 'in.ply'), Buffer.concat([header, rows]));
        const inH = await fs.promises.open(path.join(dir, 'in.ply'), 'r');
        const w3 = [];
        await host.compressPlyFile(inH, { write: async (d) => { w3.push(Buffer.from(d.buffer, d.byteOffset, d.byteLength)); } },
            actionsOf(c));
        await inH.close();
        r.file = w3.length === 4 && ['header', 'chunk', 'vertex', 'sh'].every((k, i) => w3[i].equals(bytes(arr(`${c}_${k}`))));
        // real FileHandles: the streamed writers (the arrays written at offsets as they leave HBM),
        // into a file that held longer content and at a handle position past 0
        const want = Buffer.concat(['header', 'chunk', 'vertex', 'sh'].map(k => bytes(arr(`${c}_${k}`))));
        const inH2 = await fs.promises.open(path.join(dir, 'in.ply'), 'r');
        const outP = path.join(dir, 'out.compressed.ply');
        fs.writeFileSync(outP, Buffer.alloc(want.length + 4096, 7));
        let oh = await fs.promises.open(outP, fs.constants.O_WRONLY);
        await host.compressPlyFile(inH2, oh, actionsOf(c));
        await oh.close();
        await inH2.close();
        r.fileFd = fs.readFileSync(outP).equals(want);
        oh = await fs.promises.open(outP, 'w');
        await oh.write(Buffer.from('prefix'));
        await host.writeCompressedPly(oh, tableOf(c), actionsOf(c));
        await oh.write(Buffer.from('suffix'));
        await oh.close();
        r.tableFd = fs.readFileSync(outP).equals(Buffer.concat([Buffer.from('prefix'), want, Buffer.from('suffix')]));
        fs.unlinkSync(outP);
        fs.unlinkSync(path.join(dir, 'in.ply'));
        fs.rmdirSync(dir);
        out[c] = r;
    }
    console.log(JSON.stringify(out));
})().catch((e) => { console.error(e); process.exit(1); });
