'use strict';
// Node host: tables whose columns are not float32 (tests/golden/typed_columns.*, the reference's
// own outputs): processDataTable (the processed table and the caller's table afterwards),
// writeCompressedPly with the actions in the same call, transform() and generateOrdering on the
// typed columns, and writeSog's textures + meta + draws (sogTextures).  Prints one JSON object.
const fs = require('fs');
const path = require('path');

const host = require(path.join(__dirname, '..', '..', 'splat-transform_amd', 'js'));
const GOLDEN = path.join(__dirname, '..', 'golden');

const CTOR = { f4: Float32Array, f8: Float64Array, u4: Uint32Array, i4: Int32Array, u1: Uint8Array, i1: Int8Array,
    u2: Uint16Array, i2: Int16Array };
const man = JSON.parse(fs.readFileSync(path.join(GOLDEN, 'typed_columns.json'), 'utf8'));
const blob = fs.readFileSync(path.join(GOLDEN, 'typed_columns.bin'));
const arr = (k) => {
    const a = man.arrays[k];
    const ctor = CTOR[a.dtype];
    const copy = Buffer.from(blob.subarray(a.offset, a.offset + a.nbytes));
    return new ctor(copy.buffer, copy.byteOffset, a.nbytes / ctor.BYTES_PER_ELEMENT);
};
const bytes = a => Buffer.from(a.buffer, a.byteOffset, a.byteLength);
const sameBytes = (a, b) => a.constructor === b.constructor && a.length === b.length && bytes(a).equals(bytes(b));
const actionsOf = c => man.meta[`${c}_actions`].map(a => (Array.isArray(a.value)
    ? Object.assign({}, a, { value: { x: a.value[0], y: a.value[1], z: a.value[2] } }) : a));
const tableOf = p => new host.DataTable(man.meta[`${p}columns`].map(n => new host.Column(n, arr(`${p}${n}`))));

// mulberry32 (make_golden.js): the fixtures' Math.random stream
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

(async () => {
    const out = {};
    for (const c of man.meta.cases) {
        const r = {};
        const input = tableOf(`${c}_in_`);
        const res = host.processDataTable(input, actionsOf(c));
        r.names = JSON.stringify(res.columns.map(col => col.name)) === JSON.stringify(man.meta[`${c}_out_columns`]);
        r.table = res.columns.every(col => sameBytes(col.data, arr(`${c}_out_${col.name}`)));
        r.after = input.columns.every(col => sameBytes(col.data, arr(`${c}_after_${col.name}`)));
        const writes = [];
        await host.writeCompressedPly({ write: async (d) => { writes.push(Buffer.from(d.buffer, d.byteOffset, d.byteLength)); } },
            tableOf(`${c}_in_`), actionsOf(c));
        r.writes = writes.length === 4 && ['header', 'chunk', 'vertex', 'sh'].every((k, i) => writes[i].equals(bytes(arr(`${c}_${k}`))));
        if (man.meta[`${c}_sog`]) {
            const ref = man.meta[`${c}_sog`];
            const rnd = mulberry32(ref.seed);
            const saved = Math.random;
            let count = 0;
            Math.random = () => { count++; return rnd(); };
            host.resetRandomStream();  // this case's stream starts here (make_golden.js seeds per case)
            let s;
            try {
                s = await host.sogTextures(tableOf(`${c}_sog_in_`), ref.iters);
            } finally {
                Math.random = saved;
            }
            r.sog_draws = s.used === ref.draws;
            r.sog_textures = ['means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels']
                .every(k => Buffer.from(s.textures[k]).equals(bytes(arr(`${c}_sog_${k}`))));
            r.sog_means = JSON.stringify(s.meansMins) === JSON.stringify(ref.meta.means.mins) &&
                JSON.stringify(s.meansMaxs) === JSON.stringify(ref.meta.means.maxs);
            r.sog_codebooks = JSON.stringify(Array.from(s.scalesCodebook)) === JSON.stringify(ref.meta.scales.codebook) &&
                JSON.stringify(Array.from(s.sh0Codebook)) === JSON.stringify(ref.meta.sh0.codebook) &&
                JSON.stringify(Array.from(s.shNCodebook)) === JSON.stringify(ref.meta.shN.codebook);
        }
        out[c] = r;
    }
    // transform() of the typed table alone (the f64 case's first action ran before its filter)
    {
        const t = tableOf('f64_in_');
        const a = actionsOf('f64')[0];
        host.transform(t, { x: 0, y: 0, z: 0 }, host.quatFromEuler(a.value.x, a.value.y, a.value.z), 1);
        out.transform_f64 = t.columns.every(col => sameBytes(col.data, arr(`f64_after_${col.name}`)));
    }
    console.log(JSON.stringify(out));
})().catch((e) => { console.error(e); process.exit(1); });
