'use strict';
// TEST INFRASTRUCTURE ONLY: generates tests/golden/*.{json,bin}.
//
// Runs the reference's own hot-path modules (type-erased into $ST_REF_JS by
// build_ref.py, never committed) on small synthetic inputs and records
// inputs + outputs as fixture vectors.  Math.random is replaced by a seeded
// mulberry32 stream per case; the number of draws each call consumed is
// recorded so the port can replay the identical stream.
//
//   python3 tests/golden/gen/build_ref.py && node tests/golden/gen/make_golden.js
//
// Reference call sites exercised:
//   transform.ts:12-65 via process.ts:64-145   rotate-sh.ts:46-189
//   ordering.ts:4-110                           compressed-chunk.ts:44-180
//   write-compressed-ply.ts:31-115              k-means.ts:137-201, kd-tree.ts:9-100
//   write-sog.ts:56-99 (cluster1d), :110-370   process.ts:47-61,84-95 (filterNaN)
//   index.ts:158-210 (combine)                  utils/math.ts:1

const fs = require('fs');
const path = require('path');

const REF = process.env.ST_REF_JS || '/tmp/st_ref_js';
const OUT = process.env.ST_GOLDEN_OUT || path.join(__dirname, '..');
const only = process.argv.slice(2);

const { Column, DataTable } = require(path.join(REF, 'data-table.js'));
const { generateOrdering } = require(path.join(REF, 'ordering.js'));
const { processDataTable } = require(path.join(REF, 'process.js'));
const { RotateSH } = require(path.join(REF, 'utils/rotate-sh.js'));
const { sigmoid } = require(path.join(REF, 'utils/math.js'));
// every kmeans() call writeSog makes can be recorded (sog65k): the k-means module's export is
// wrapped BEFORE write-sog.js binds it; the wrapper calls the reference function unchanged
const kmeansModule = require(path.join(REF, 'utils/k-means.js'));
const kmeansCalls = [];
let recordKmeans = false;
{
    const origKmeans = kmeansModule.kmeans;
    kmeansModule.kmeans = async (points, k, iters, device) => {
        const drawsBefore = drawCount;
        const res = await origKmeans(points, k, iters, device);
        if (recordKmeans) {
            kmeansCalls.push({ n: points.numRows, d: points.numColumns, k, iters, drawsBefore, drawsAfter: drawCount,
                centroids: res.centroids.columns.map(c => Float32Array.from(c.data)), labels: Uint32Array.from(res.labels) });
        }
        return res;
    };
}
const { kmeans } = kmeansModule;
const { writeCompressedPly } = require(path.join(REF, 'writers/write-compressed-ply.js'));
const { writeSog, cluster1d } = require(path.join(REF, 'writers/write-sog.js'));
const { combine } = require(path.join(REF, 'index.js'));
const { readPly } = require(path.join(REF, 'readers/read-ply.js'));
const { isCompressedPly, decompressPly } = require(path.join(REF, 'readers/decompress-ply.js'));
const pc = require(path.join(REF, '__stubs/playcanvas.js'));

// ---------------------------------------------------------------------------
// deterministic generators
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

class Gen {
    constructor(seed) { this.u = mulberry32(seed); this.spare = null; }
    uniform(a, b) { return a + (b - a) * this.u(); }
    normal(mu = 0, sigma = 1) {
        if (this.spare !== null) { const s = this.spare; this.spare = null; return mu + sigma * s; }
        let u1 = this.u(); while (u1 === 0) u1 = this.u();
        const u2 = this.u();
        const r = Math.sqrt(-2 * Math.log(u1));
        this.spare = r * Math.sin(2 * Math.PI * u2);
        return mu + sigma * r * Math.cos(2 * Math.PI * u2);
    }
    int(n) { return Math.floor(this.u() * n); }
}

// Math.random replacement with draw counting
let drawCount = 0;
const seedRandom = (seed) => {
    const r = mulberry32(seed);
    drawCount = 0;
    Math.random = () => { drawCount++; return r(); };
};

const quiet = async (fn) => {
    const log = console.log, w = process.stdout.write;
    console.log = () => {};
    process.stdout.write = () => true;
    try { return await fn(); } finally { console.log = log; process.stdout.write = w; }
};

// ---------------------------------------------------------------------------
// fixture container: <name>.json manifest + <name>.bin blob (little endian)
class Fixture {
    constructor(name) { this.name = name; this.arrays = {}; this.chunks = []; this.offset = 0; this.meta = {}; }
    add(key, arr, shape) {
        const dtype = {
            Float32Array: 'f4', Float64Array: 'f8', Uint32Array: 'u4', Int32Array: 'i4',
            Uint8Array: 'u1', Int8Array: 'i1', Uint16Array: 'u2', Int16Array: 'i2'
        }[arr.constructor.name];
        if (!dtype) throw new Error(`bad array type for ${key}`);
        const buf = Buffer.from(arr.buffer, arr.byteOffset, arr.byteLength);
        const pad = (8 - (this.offset % 8)) % 8;
        if (pad) { this.chunks.push(Buffer.alloc(pad)); this.offset += pad; }
        this.arrays[key] = { dtype, shape: shape || [arr.length], offset: this.offset, nbytes: buf.length };
        this.chunks.push(Buffer.from(buf));
        this.offset += buf.length;
    }
    save() {
        fs.writeFileSync(path.join(OUT, `${this.name}.bin`), Buffer.concat(this.chunks));
        fs.writeFileSync(path.join(OUT, `${this.name}.json`), JSON.stringify({
            generator: 'tests/golden/gen/make_golden.js (reference modules type-erased by build_ref.py)',
            reference: '@playcanvas/splat-transform 0.10.1 @ /root/reference',
            meta: this.meta,
            arrays: this.arrays
        }, null, 1));
        const kb = (this.offset / 1024).toFixed(1);
        process.stderr.write(`  ${this.name}: ${Object.keys(this.arrays).length} arrays, ${kb} KiB\n`);
    }
}

const shNames = (n) => new Array(n).fill('').map((_, i) => `f_rest_${i}`);

// standard 3DGS column order (read-ply column order of a typical file)
const gsColumnNames = (shCoeffs) => [
    'x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2',
    ...shNames(shCoeffs * 3), 'opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3'
];

// synthetic splats following SURVEY.md §8d distributions
const makeSplats = (n, shCoeffs, seed, opts = {}) => {
    const g = new Gen(seed);
    const names = gsColumnNames(shCoeffs);
    const cols = {};
    names.forEach((nm) => { cols[nm] = new Float32Array(n); });
    const cube = opts.cubeFrac || 0;
    for (let i = 0; i < n; ++i) {
        if (g.u() < cube) {
            cols.x[i] = 1 + g.uniform(0, 1e-3); cols.y[i] = -2 + g.uniform(0, 1e-3); cols.z[i] = 3 + g.uniform(0, 1e-3);
        } else {
            cols.x[i] = g.normal(0, 10); cols.y[i] = g.normal(0, 10); cols.z[i] = g.normal(0, 10);
        }
        for (let c = 0; c < 3; ++c) cols[`f_dc_${c}`][i] = g.normal(0, 1);
        for (let c = 0; c < shCoeffs * 3; ++c) cols[`f_rest_${c}`][i] = g.normal(0, 0.1);
        cols.opacity[i] = g.normal(0, 2);
        for (let c = 0; c < 3; ++c) cols[`scale_${c}`][i] = g.uniform(-7, -2);
        for (let c = 0; c < 4; ++c) cols[`rot_${c}`][i] = g.normal(0, 1);
    }
    return { names, cols };
};

// transcendental-free splats (sog65k): every value is made of mulberry32 draws with + - * only,
// so numpy reproduces the table bit for bit (tests/golden_io.py: bell_splats).  228 draws per row:
// cube flag, 4 per x/y/z, f_dc, f_rest, opacity, rot (Irwin-Hall sum of 4 draws), 1 per scale.
const makeBellSplats = (n, shCoeffs, seed, cubeFrac) => {
    const u = mulberry32(seed);
    const bell = (sigma) => ((((u() + u()) + u()) + u()) - 2) * sigma;
    const names = gsColumnNames(shCoeffs);
    const cols = {};
    names.forEach((nm) => { cols[nm] = new Float32Array(n); });
    const off = [1, -2, 3];
    for (let i = 0; i < n; ++i) {
        const cube = u() < cubeFrac;
        ['x', 'y', 'z'].forEach((a, j) => {
            const v = bell(17.32);
            cols[a][i] = cube ? off[j] + (v + 34.64) * 1e-5 : v;
        });
        for (let c = 0; c < 3; ++c) cols[`f_dc_${c}`][i] = bell(1.732);
        for (let c = 0; c < shCoeffs * 3; ++c) cols[`f_rest_${c}`][i] = bell(0.1732);
        cols.opacity[i] = bell(3.464);
        for (let c = 0; c < 3; ++c) cols[`scale_${c}`][i] = -7 + 5 * u();
        for (let c = 0; c < 4; ++c) cols[`rot_${c}`][i] = bell(1.732);
    }
    return { names, cols };
};

const sha256 = (arr) => require('crypto').createHash('sha256')
    .update(Buffer.from(arr.buffer, arr.byteOffset, arr.byteLength)).digest('hex');

const toTable = (names, cols) => new DataTable(names.map(nm => new Column(nm, cols[nm].slice())));

const addTable = (fx, prefix, table) => {
    fx.meta[`${prefix}columns`] = table.columns.map(c => c.name);
    table.columns.forEach((c) => { fx.add(`${prefix}${c.name}`, c.data); });
};

// ---------------------------------------------------------------------------
const cases = {};

cases.mathfns = () => {
    const fx = new Fixture('mathfns');
    const g = new Gen(7);
    const xs = [];
    const specials = [0, -0, 1, -1, 0.5, -0.5, 2, 1e-10, -1e-10, 1e-300, 5e-324, 709.78, 709.79, -745.1, -745.2,
        700, -700, 88.7, -103.9, 20, -20, 1e308, -1e308, Infinity, -Infinity, NaN, Math.LN2, -Math.LN2,
        0.34657359027997264, 1.0397207708399179, 2.2250738585072014e-308];
    specials.forEach(v => xs.push(v));
    for (let i = 0; i < 3000; ++i) xs.push(Math.fround(g.uniform(-20, 20)));
    for (let i = 0; i < 3000; ++i) xs.push(Math.fround(g.normal(0, 2)));
    for (let i = 0; i < 4000; ++i) xs.push(g.uniform(-745, 709.7));
    for (let i = 0; i < 4000; ++i) xs.push(Math.fround(g.uniform(-7, -2)));
    for (let i = 0; i < 4000; ++i) xs.push(Math.fround(g.normal(0, 10)));
    for (let i = 0; i < 2000; ++i) xs.push(Math.pow(2, g.uniform(-1060, 1020)) * (g.u() < 0.5 ? -1 : 1));
    const x = new Float64Array(xs);
    const ex = x.map(v => Math.exp(v));
    const lg = x.map(v => Math.log(v));
    const lga = x.map(v => Math.log(Math.abs(v) + 1));
    const sg = x.map(v => sigmoid(v));
    const lt = x.map(v => Math.sign(v) * Math.log(Math.abs(v) + 1));
    const sc05 = x.map(v => Math.log(Math.exp(v) * 0.5));
    const sc2 = x.map(v => Math.log(Math.exp(v) * 2));
    fx.add('x', x); fx.add('exp', ex); fx.add('log', lg); fx.add('log1abs', lga); fx.add('sigmoid', sg);
    fx.add('logtransform', lt); fx.add('logexp_s05', sc05); fx.add('logexp_s2', sc2);
    fx.save();
};

const ACTION_LISTS = [
    [{ kind: 'rotate', value: new pc.Vec3(0, 45, 0) }],
    [{ kind: 'scale', value: 0.5 }, { kind: 'translate', value: new pc.Vec3(0, 0, 10) }],
    [{ kind: 'rotate', value: new pc.Vec3(10, 20, 30) }, { kind: 'scale', value: 2 }, { kind: 'translate', value: new pc.Vec3(-1, 2.5, 3) }],
    [{ kind: 'rotate', value: new pc.Vec3(90, 0, 0) }],
    [{ kind: 'rotate', value: new pc.Vec3(-30.5, 170, 45.25) }],
    [{ kind: 'translate', value: new pc.Vec3(0.1, -0.2, 0.3) }]
];

const injectEdges = (cols, names, shCoeffs) => {
    // rows 0..9 carry edge values
    cols.x[0] = NaN; cols.y[1] = Infinity; cols.z[2] = -0;
    cols.x[3] = 1e30; cols.y[3] = -1e30; cols.z[3] = 3e-39;
    for (let c = 0; c < 4; ++c) cols[`rot_${c}`][4] = 0;
    cols.rot_0[5] = NaN;
    cols.scale_0[6] = Infinity; cols.scale_1[6] = -Infinity; cols.scale_2[6] = NaN;
    cols.scale_0[7] = 80; cols.scale_1[7] = -200;
    if (shCoeffs > 0) {
        cols.f_rest_0[8] = NaN;
        cols.f_rest_1[8] = -0;
        cols[`f_rest_${shCoeffs * 3 - 1}`][9] = Infinity;
        for (let c = 0; c < shCoeffs * 3; ++c) cols[`f_rest_${c}`][7] = -0;
    }
    cols.opacity[9] = -0;
};

cases.transform = () => {
    const fx = new Fixture('transform');
    fx.meta.actions = ACTION_LISTS.map(list => list.map(a => ({
        kind: a.kind, value: (typeof a.value === 'number') ? a.value : [a.value.x, a.value.y, a.value.z]
    })));
    // per-action host parameters (Quat, Mat4 f32 data, RotateSH matrices as f64)
    ACTION_LISTS.forEach((list, li) => {
        list.forEach((a, ai) => {
            let t = pc.Vec3.ZERO, r = pc.Quat.IDENTITY, s = 1;
            if (a.kind === 'translate') t = a.value;
            if (a.kind === 'rotate') r = new pc.Quat().setFromEulerAngles(a.value.x, a.value.y, a.value.z);
            if (a.kind === 'scale') s = a.value;
            const mat = new pc.Mat4().setTRS(t, r, new pc.Vec3(s, s, s));
            const mat3 = new pc.Mat3().setFromQuat(r);
            const rsh = new RotateSH(mat3);
            const cols = new Float64Array(15 * 15);
            for (let j = 0; j < 15; ++j) {
                const e = new Array(15).fill(0); e[j] = 1;
                const res = e.slice();
                rsh.apply(res);
                for (let i = 0; i < 15; ++i) cols[i * 15 + j] = res[i];
            }
            fx.add(`p${li}_${ai}_quat`, new Float64Array([r.x, r.y, r.z, r.w]));
            fx.add(`p${li}_${ai}_mat4`, mat.data.slice());
            fx.add(`p${li}_${ai}_mat3`, mat3.data.slice());
            fx.add(`p${li}_${ai}_shrot`, cols, [15, 15]);
        });
    });
    [0, 1, 2, 3].forEach((band) => {
        const shCoeffs = [0, 3, 8, 15][band];
        const n = band === 3 ? 768 : 384;
        const { names, cols } = makeSplats(n, shCoeffs, 100 + band);
        injectEdges(cols, names, shCoeffs);
        addTable(fx, `b${band}_in_`, toTable(names, cols));
        ACTION_LISTS.forEach((list, li) => {
            const table = toTable(names, cols);
            const out = processDataTable(table, list);
            const touched = out.columns.filter(c => /^(x|y|z|rot_\d|scale_\d|f_rest_\d+)$/.test(c.name));
            touched.forEach((c) => fx.add(`b${band}_a${li}_${c.name}`, c.data));
            // untouched columns must come back unchanged
            out.columns.forEach((c) => {
                if (touched.indexOf(c) < 0) {
                    const a = new Uint32Array(c.data.buffer), b = new Uint32Array(cols[c.name].buffer);
                    for (let i = 0; i < a.length; ++i) if (a[i] !== b[i]) throw new Error(`untouched ${c.name} changed`);
                }
            });
        });
    });
    fx.save();
};

const orderingInputs = () => {
    const out = [];
    const g = new Gen(31);
    const mk = (n, f) => { const x = new Float32Array(n), y = new Float32Array(n), z = new Float32Array(n); for (let i = 0; i < n; ++i) f(i, x, y, z); return { x, y, z }; };
    out.push(['nested_cube', mk(20000, (i, x, y, z) => {
        if (g.u() < 0.1) { x[i] = 1 + g.uniform(0, 1e-4); y[i] = 2 + g.uniform(0, 1e-4); z[i] = 3 + g.uniform(0, 1e-4); } else { x[i] = g.normal(0, 10); y[i] = g.normal(0, 10); z[i] = g.normal(0, 10); }
    })]);
    out.push(['identical_bucket', mk(3000, (i, x, y, z) => {
        if (i % 10 === 3) { x[i] = 0.5; y[i] = 0.25; z[i] = -0.125; } else { x[i] = g.normal(0, 1); y[i] = g.normal(0, 1); z[i] = g.normal(0, 1); }
    })]);
    out.push(['nan_first', mk(1000, (i, x, y, z) => { x[i] = i === 0 ? NaN : g.normal(); y[i] = g.normal(); z[i] = g.normal(); })]);
    out.push(['nan_later', mk(1000, (i, x, y, z) => { x[i] = i === 5 ? NaN : g.normal(); y[i] = i === 17 ? NaN : g.normal(); z[i] = g.normal(); })]);
    out.push(['inf', mk(1000, (i, x, y, z) => { x[i] = g.normal(); y[i] = i === 400 ? -Infinity : g.normal(); z[i] = g.normal(); })]);
    out.push(['line', mk(2000, (i, x, y, z) => { x[i] = g.uniform(-5, 5); y[i] = 0; z[i] = 7; })]);
    out.push(['empty', mk(0, () => {})]);
    out.push(['one', mk(1, (i, x, y, z) => { x[i] = 1; y[i] = 2; z[i] = 3; })]);
    out.push(['two', mk(2, (i, x, y, z) => { x[i] = 2 - i; y[i] = i; z[i] = 0; })]);
    out.push(['deep_nest', mk(6000, (i, x, y, z) => {
        const r = g.u();
        if (r < 0.4) { x[i] = 5 + g.uniform(0, 1e-6); y[i] = 5 + g.uniform(0, 1e-6); z[i] = 5 + g.uniform(0, 1e-6); }
        else if (r < 0.6) { x[i] = 5 + Math.floor(g.u() * 4) * 1e-7; y[i] = 5; z[i] = 5 + Math.floor(g.u() * 3) * 1e-7; }
        else { x[i] = g.normal(0, 100); y[i] = g.normal(0, 100); z[i] = g.normal(0, 100); }
    })]);
    out.push(['bucket_256_257', mk(4000, (i, x, y, z) => {
        if (i < 256) { x[i] = -3; y[i] = -3; z[i] = -3; }
        else if (i < 513) { x[i] = 3; y[i] = 3; z[i] = 3; }
        else { x[i] = g.uniform(-3, 3); y[i] = g.uniform(-3, 3); z[i] = g.uniform(-3, 3); }
    })]);
    out.push(['grid_dups', mk(5000, (i, x, y, z) => { x[i] = Math.floor(g.u() * 6); y[i] = Math.floor(g.u() * 5) * 0.5; z[i] = Math.floor(g.u() * 4) - 2; })]);
    out.push(['neg_zero', mk(600, (i, x, y, z) => { x[i] = (i & 1) ? -0 : 0; y[i] = g.normal(); z[i] = (i % 3) ? 0 : -0; })]);
    return out;
};

cases.ordering = () => {
    const fx = new Fixture('ordering');
    const names = [];
    orderingInputs().forEach(([name, { x, y, z }]) => {
        names.push(name);
        const dt = new DataTable([new Column('x', x), new Column('y', y), new Column('z', z)].filter(() => true));
        const idx = new Uint32Array(x.length);
        for (let i = 0; i < idx.length; ++i) idx[i] = i;
        if (x.length > 0) quiet(() => generateOrdering(dt, idx));
        fx.add(`${name}_x`, x); fx.add(`${name}_y`, y); fx.add(`${name}_z`, z); fx.add(`${name}_order`, idx);
    });
    fx.meta.cases = names;
    fx.save();
};

const captureHandle = () => {
    const writes = [];
    return { writes, handle: { write: async (d) => { writes.push(Buffer.from(d.buffer, d.byteOffset, d.byteLength)); } } };
};

cases.compressed_ply = async () => {
    const fx = new Fixture('compressed_ply');
    const specs = [['sh3', 3000, 15, 0.06], ['sh0', 700, 0, 0.0], ['sh1', 1100, 3, 0.3], ['sh2', 600, 8, 0.0]];
    fx.meta.cases = specs.map(s => s[0]);
    for (const [name, n, shc, cube] of specs) {
        const { names, cols } = makeSplats(n, shc, 200 + n, { cubeFrac: cube });
        if (name === 'sh3') {
            // chunk 3 (rows by Morton order unknown, so poison raw rows) : edge values
            cols.scale_0[10] = Infinity; cols.scale_1[11] = -Infinity; cols.scale_2[12] = 25;
            cols.rot_0[13] = 0; cols.rot_1[13] = 0; cols.rot_2[13] = 0; cols.rot_3[13] = 0;
            cols.opacity[14] = 60; cols.opacity[15] = -60;
            cols.f_rest_0[16] = 4.5; cols.f_rest_1[16] = -4.5; cols.f_rest_2[16] = 3.99;
            cols.rot_0[17] = -0.5; cols.rot_1[17] = 0.5; cols.rot_2[17] = -0.5; cols.rot_3[17] = 0.5;
            cols.f_dc_0[18] = NaN;
        }
        const table = toTable(names, cols);
        addTable(fx, `${name}_in_`, table);
        const { writes, handle } = captureHandle();
        await quiet(() => writeCompressedPly(handle, table));
        if (writes.length !== 4) throw new Error('expected 4 writes');
        const u8 = (b) => new Uint8Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.length));
        fx.add(`${name}_header`, u8(writes[0]));
        fx.add(`${name}_chunk`, new Float32Array(u8(writes[1]).buffer));
        fx.add(`${name}_vertex`, new Uint32Array(u8(writes[2]).buffer));
        fx.add(`${name}_sh`, u8(writes[3]));
    }
    fx.save();
};

cases.kmeans = async () => {
    const fx = new Fixture('kmeans');
    const g = new Gen(41);
    const specs = [];
    const mkCols = (n, d, f) => { const c = []; for (let j = 0; j < d; ++j) c.push(new Float32Array(n)); for (let i = 0; i < n; ++i) f(i, c); return c; };
    specs.push(['d1_normal', 256, 5, 11, mkCols(20000, 1, (i, c) => { c[0][i] = g.normal(); })]);
    specs.push(['d1_ints', 256, 4, 12, mkCols(5000, 1, (i, c) => { c[0][i] = Math.floor(g.u() * 41); })]);
    specs.push(['d1_halves', 64, 6, 13, mkCols(3000, 1, (i, c) => { c[0][i] = Math.floor(g.u() * 300) * 0.5 - 20; })]);
    specs.push(['d45_normal', 256, 3, 14, mkCols(3000, 45, (i, c) => { for (let j = 0; j < 45; ++j) c[j][i] = g.normal(0, 0.1); })]);
    const base = mkCols(300, 45, (i, c) => { for (let j = 0; j < 45; ++j) c[j][i] = g.normal(0, 0.1); });
    specs.push(['d45_dups', 512, 3, 15, mkCols(2000, 45, (i, c) => { const r = g.int(300); for (let j = 0; j < 45; ++j) c[j][i] = base[j][r]; })]);
    specs.push(['d3_grid', 64, 4, 16, mkCols(4000, 3, (i, c) => { for (let j = 0; j < 3; ++j) c[j][i] = Math.floor(g.u() * 5); })]);
    specs.push(['d9_normal', 1024, 2, 17, mkCols(2500, 9, (i, c) => { for (let j = 0; j < 9; ++j) c[j][i] = g.normal(0, 0.3); })]);
    specs.push(['n_lt_k', 256, 3, 18, mkCols(100, 2, (i, c) => { c[0][i] = g.normal(); c[1][i] = g.normal(); })]);
    specs.push(['d24_mixed', 300, 3, 19, mkCols(1500, 24, (i, c) => { for (let j = 0; j < 24; ++j) c[j][i] = (i % 7 === 0) ? 0.25 : g.normal(0, 0.2); })]);
    fx.meta.cases = [];
    for (const [name, k, iters, seed, cols] of specs) {
        const table = new DataTable(cols.map((c, j) => new Column(`c${j}`, c)));
        seedRandom(seed);
        const { centroids, labels } = await quiet(() => kmeans(table, k, iters));
        fx.meta.cases.push({ name, k, iters, seed, n: cols[0].length, d: cols.length, draws: drawCount });
        cols.forEach((c, j) => fx.add(`${name}_p${j}`, c));
        centroids.columns.forEach((c, j) => fx.add(`${name}_c${j}`, new Float32Array(c.data)));
        fx.add(`${name}_labels`, Uint32Array.from(labels));
    }
    // cluster1d (write-sog.ts:56-99): 3 columns flattened column-major, k=256
    const c1 = mkCols(4000, 3, (i, c) => { c[0][i] = g.uniform(-7, -2); c[1][i] = g.uniform(-7, -2); c[2][i] = (i % 5 === 0) ? -4 : g.uniform(-7, -2); });
    const t1 = new DataTable(c1.map((c, j) => new Column(`scale_${j}`, c)));
    seedRandom(99);
    const r1 = await quiet(() => cluster1d(t1, 5));
    fx.meta.cluster1d = { seed: 99, iters: 5, n: 4000, draws: drawCount };
    c1.forEach((c, j) => fx.add(`cluster1d_p${j}`, c));
    fx.add('cluster1d_centroids', new Float32Array(r1.centroids.getColumn(0).data));
    r1.labels.columns.forEach((c, j) => fx.add(`cluster1d_l${j}`, c.data));
    fx.save();
};

const readRGBA = (file) => {
    const b = fs.readFileSync(file);
    if (b.toString('ascii', 0, 4) !== 'RGBA') throw new Error('bad stub texture');
    return { w: b.readUInt32LE(4), h: b.readUInt32LE(8), data: new Uint8Array(b.buffer.slice(b.byteOffset + 16, b.byteOffset + b.length)) };
};

cases.sog = async () => {
    const fx = new Fixture('sog');
    const specs = [['sh3', 6000, 15, 2, 21, 0.05], ['sh0', 3000, 0, 3, 22, 0.05], ['sh1', 2048, 3, 2, 23, 0.0], ['sh2', 2100, 8, 2, 24, 0.1]];
    fx.meta.cases = [];
    for (const [name, n, shc, iters, seed, cube] of specs) {
        const { names, cols } = makeSplats(n, shc, 300 + n, { cubeFrac: cube });
        if (name === 'sh3') { cols.rot_0[3] = 0; cols.rot_1[3] = 0; cols.rot_2[3] = 0; cols.rot_3[3] = 0; cols.x[4] = 0; cols.y[4] = -0; }
        const table = toTable(names, cols);
        addTable(fx, `${name}_in_`, table);
        const dir = fs.mkdtempSync('/tmp/st_sog_');
        const metaPath = path.join(dir, 'meta.json');
        const fh = await fs.promises.open(metaPath, 'w');
        seedRandom(seed);
        await quiet(() => writeSog(fh, table, metaPath, iters, 'cpu'));
        await fh.close();
        const meta = JSON.parse(fs.readFileSync(metaPath, 'utf8'));
        fx.meta.cases.push({ name, n, iters, seed, draws: drawCount, meta });
        const files = ['means_l', 'means_u', 'quats', 'scales', 'sh0'].concat(shc ? ['shN_centroids', 'shN_labels'] : []);
        files.forEach((f) => {
            const t = readRGBA(path.join(dir, `${f}.webp`));
            fx.add(`${name}_${f}`, t.data, [t.h, t.w, 4]);
        });
        fs.rmSync ? fs.rmSync(dir, { recursive: true }) : fs.rmdirSync(dir, { recursive: true });
    }
    fx.save();
};

// Tables whose columns are not float32 -- a PLY with `double` properties, and integer ones:
// the reference reads every column through getRow as numbers and stores through setRow
// (data-table.ts:63-76), so transform, ordering, the compressed-PLY writer and writeSog take
// them.  Per case: processDataTable + writeCompressedPly (as process_chain: input, processed
// table, the input afterwards, the four writes) and writeSog of the input (textures + meta).
cases.typed_columns = async () => {
    const fx = new Fixture('typed_columns');
    // values in each column's own type: float64 columns hold unrounded numbers, integer columns
    // the truncated (scaled) values a TypedArray store keeps
    const makeTyped = (n, shCoeffs, seed, typeOf, scaleOf, cubeFrac) => {
        const g = new Gen(seed);
        const names = gsColumnNames(shCoeffs);
        const cols = {};
        names.forEach((nm) => { cols[nm] = new (typeOf(nm))(n); });
        const put = (nm, i, v) => { cols[nm][i] = v * scaleOf(nm); };
        for (let i = 0; i < n; ++i) {
            if (g.u() < cubeFrac) {
                put('x', i, 1 + g.uniform(0, 1e-3)); put('y', i, -2 + g.uniform(0, 1e-3)); put('z', i, 3 + g.uniform(0, 1e-3));
            } else {
                put('x', i, g.normal(0, 10)); put('y', i, g.normal(0, 10)); put('z', i, g.normal(0, 10));
            }
            for (let c = 0; c < 3; ++c) put(`f_dc_${c}`, i, g.normal(0, 1));
            for (let c = 0; c < shCoeffs * 3; ++c) put(`f_rest_${c}`, i, g.normal(0, 0.1));
            put('opacity', i, g.normal(0, 2));
            for (let c = 0; c < 3; ++c) put(`scale_${c}`, i, g.uniform(-7, -2));
            for (let c = 0; c < 4; ++c) put(`rot_${c}`, i, g.normal(0, 1));
        }
        return { names, cols };
    };
    const V = (x, y, z) => new pc.Vec3(x, y, z);
    const mixedType = (nm) => ({ x: Float64Array, y: Int16Array, z: Int32Array, rot_0: Float64Array, opacity: Float64Array,
        scale_0: Int8Array, scale_1: Int8Array, scale_2: Float64Array, f_dc_2: Uint16Array, f_rest_1: Float64Array,
        f_rest_4: Float64Array, f_rest_7: Uint8Array, f_rest_8: Int8Array }[nm] || Float32Array);
    const mixedScale = (nm) => ({ y: 100, z: 1000, f_dc_2: 1000, f_rest_7: 300, f_rest_8: 300 }[nm] || 1);
    const specs = [
        ['f64', () => makeTyped(1500, 15, 951, () => Float64Array, () => 1, 0.2),
            [{ kind: 'rotate', value: V(0, 45, 0) }, { kind: 'filterNaN' }], 2500],
        ['mixed', () => makeTyped(1400, 3, 952, mixedType, mixedScale, 0.25),
            [{ kind: 'translate', value: V(1.5, -2.25, 3) }, { kind: 'scale', value: 2 }, { kind: 'filterNaN' }], 2500],
        ['f64_sh1_bands', () => makeTyped(1900, 8, 953, () => Float64Array, () => 1, 0.0),
            [{ kind: 'filterBands', value: 1 }, { kind: 'rotate', value: V(30, -60, 10) },
                { kind: 'filterByValue', columnName: 'opacity', comparator: 'gt', value: -1 }], 0],
    ];
    fx.meta.cases = specs.map(s => s[0]);
    for (const [name, make, acts, sogN] of specs) {
        const { names, cols } = make();
        if (name === 'f64') { cols.x[10] = NaN; cols.f_rest_40[11] = Infinity; cols.rot_2[12] = -Infinity; }
        const table = toTable(names, cols);
        fx.meta[`${name}_actions`] = acts.map(a => (a.value && a.value.x !== undefined)
            ? Object.assign({}, a, { value: [a.value.x, a.value.y, a.value.z] }) : a);
        fx.meta[`${name}_in_types`] = table.columns.map(c => c.dataType);
        addTable(fx, `${name}_in_`, table);
        const out = processDataTable(table, acts);
        fx.meta[`${name}_out_types`] = out.columns.map(c => c.dataType);
        addTable(fx, `${name}_out_`, out);
        addTable(fx, `${name}_after_`, table);
        const { writes, handle } = captureHandle();
        await quiet(() => writeCompressedPly(handle, out));
        const u8 = (b) => new Uint8Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.length));
        fx.add(`${name}_header`, u8(writes[0]));
        fx.add(`${name}_chunk`, new Float32Array(u8(writes[1]).buffer));
        fx.add(`${name}_vertex`, new Uint32Array(u8(writes[2]).buffer));
        fx.add(`${name}_sh`, u8(writes[3]));
        if (!sogN) continue;
        // writeSog of a fresh table of the same types (sogN rows; iters 2)
        const st = make === specs[0][1] ? makeTyped(sogN, 15, 961, () => Float64Array, () => 1, 0.05)
            : makeTyped(sogN, 3, 962, mixedType, mixedScale, 0.05);
        const stable = toTable(st.names, st.cols);
        addTable(fx, `${name}_sog_in_`, stable);
        fx.meta[`${name}_sog_in_types`] = stable.columns.map(c => c.dataType);
        const dir = fs.mkdtempSync('/tmp/st_sogt_');
        const metaPath = path.join(dir, 'meta.json');
        const fh = await fs.promises.open(metaPath, 'w');
        seedRandom(970 + sogN);
        await quiet(() => writeSog(fh, stable, metaPath, 2, 'cpu'));
        await fh.close();
        const meta = JSON.parse(fs.readFileSync(metaPath, 'utf8'));
        fx.meta[`${name}_sog`] = { n: sogN, iters: 2, seed: 970 + sogN, draws: drawCount, meta };
        ['means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels'].forEach((f) => {
            const t = readRGBA(path.join(dir, `${f}.webp`));
            fx.add(`${name}_sog_${f}`, t.data, [t.h, t.w, 4]);
        });
        fs.rmSync ? fs.rmSync(dir, { recursive: true }) : fs.rmdirSync(dir, { recursive: true });
    }
    fx.save();
};

// .sog bundle (write-sog.ts:110-140,361-366 + serialize/zip-writer.ts + crc.ts): the
// whole ZIP with a pinned clock, so the container layout, the CRC-32 of every entry
// and the raw meta.json text are fixed.  Entries hold the identity WebP stand-in's
// payload (16-byte 'RGBA' header + pixels; see build_ref.py).
cases.sog_bundle = async () => {
    const fx = new Fixture('sog_bundle');
    const specs = [['b_sh1', 2048, 3, 2, 31, 0.0], ['b_sh0', 1500, 0, 2, 32, 0.05]];
    const clock = [2024, 4, 17, 13, 37, 42];  // local time: dosTime/dosDate fixed
    fx.meta.cases = [];
    const RealDate = Date;
    for (const [name, n, shc, iters, seed, cube] of specs) {
        const { names, cols } = makeSplats(n, shc, 400 + n, { cubeFrac: cube });
        const table = toTable(names, cols);
        addTable(fx, `${name}_in_`, table);
        const dir = fs.mkdtempSync('/tmp/st_sogb_');
        const outPath = path.join(dir, 'scene.sog');
        const fh = await fs.promises.open(outPath, 'w');
        seedRandom(seed);
        global.Date = class extends RealDate { constructor(...a) { super(...(a.length ? a : clock)); } };
        try {
            await quiet(() => writeSog(fh, table, outPath, iters, 'cpu'));
        } finally {
            global.Date = RealDate;
        }
        await fh.close();
        const zip = fs.readFileSync(outPath);
        fx.meta.cases.push({ name, n, iters, seed, draws: drawCount, clock });
        fx.add(`${name}_zip`, new Uint8Array(zip.buffer, zip.byteOffset, zip.length));
        fs.rmSync ? fs.rmSync(dir, { recursive: true }) : fs.rmdirSync(dir, { recursive: true });
    }
    fx.save();
};

// PLY ingest (readers/read-ply.ts:111-191) and the compressed-PLY reader
// (readers/decompress-ply.ts:6-232): a mixed-type two-element PLY, and the
// compressed files of the compressed_ply cases read back and decompressed.
cases.ply_io = async () => {
    const fx = new Fixture('ply_io');
    const dir = fs.mkdtempSync('/tmp/st_ply_');
    const readFile = async (bytes) => {
        const p = path.join(dir, 'f.ply');
        fs.writeFileSync(p, bytes);
        const fh = await fs.promises.open(p, 'r');
        try { return await readPly(fh); } finally { await fh.close(); }
    };
    // (1) mixed property types, comments, two elements
    const g = new Gen(611);
    const props = [['float', 'x', 4], ['double', 'd', 8], ['uchar', 'u', 1], ['char', 'c', 1], ['short', 's', 2],
        ['ushort', 'us', 2], ['int', 'i', 4], ['uint', 'ui', 4], ['float', 'y', 4]];
    const nv = 1500, ne = 7;
    const header = ['ply', 'format binary_little_endian 1.0', 'comment made by make_golden.js', 'comment second',
        `element vertex ${nv}`].concat(props.map(p => `property ${p[0]} ${p[1]}`))
        .concat([`element extra ${ne}`, 'property float a', 'property uchar b', 'end_header']).join('\n') + '\n';
    const rowV = props.reduce((t, p) => t + p[2], 0), rowE = 5;
    const body = Buffer.alloc(nv * rowV + ne * rowE);
    let o = 0;
    for (let r = 0; r < nv; ++r) {
        body.writeFloatLE(g.normal(0, 10), o); o += 4;
        body.writeDoubleLE(g.normal(0, 1e6), o); o += 8;
        body.writeUInt8(g.int(256), o); o += 1;
        body.writeInt8(g.int(256) - 128, o); o += 1;
        body.writeInt16LE(g.int(65536) - 32768, o); o += 2;
        body.writeUInt16LE(g.int(65536), o); o += 2;
        body.writeInt32LE((g.int(65536) << 16) | g.int(65536), o); o += 4;
        body.writeUInt32LE(((g.int(65536) << 16) | g.int(65536)) >>> 0, o); o += 4;
        body.writeFloatLE(r === 3 ? NaN : g.normal(), o); o += 4;
    }
    for (let r = 0; r < ne; ++r) {
        body.writeFloatLE(r * 0.25, o); o += 4;
        body.writeUInt8(200 + r, o); o += 1;
    }
    const file = Buffer.concat([Buffer.from(header, 'ascii'), body]);
    fx.add('mixed_file', new Uint8Array(file.buffer, file.byteOffset, file.length));
    const ply = await readFile(file);
    fx.meta.mixed = { comments: ply.comments, elements: ply.elements.map(e => ({
        name: e.name, rows: e.dataTable.numRows,
        columns: e.dataTable.columns.map(c => [c.name, c.dataType]) })) };
    for (const e of ply.elements) for (const c of e.dataTable.columns) fx.add(`mixed_${e.name}_${c.name}`, c.data);
    // (2) the compressed PLY files of the compressed_ply fixture, read and decompressed
    const cp = JSON.parse(fs.readFileSync(path.join(OUT, 'compressed_ply.json'), 'utf8'));
    const blob = fs.readFileSync(path.join(OUT, 'compressed_ply.bin'));
    const part = (k) => { const a = cp.arrays[k]; return blob.subarray(a.offset, a.offset + a.nbytes); };
    fx.meta.compressed = [];
    for (const name of cp.meta.cases) {
        const f = Buffer.concat([part(`${name}_header`), part(`${name}_chunk`), part(`${name}_vertex`), part(`${name}_sh`)]);
        const cply = await readFile(f);
        const ok = isCompressedPly(cply);
        fx.meta.compressed.push({ name, isCompressed: ok });
        if (!ok) continue;
        const out = decompressPly(cply);
        fx.meta[`${name}_columns`] = out.columns.map(c => c.name);
        for (const c of out.columns) fx.add(`${name}_dec_${c.name}`, c.data);
    }
    fs.rmSync ? fs.rmSync(dir, { recursive: true }) : fs.rmdirSync(dir, { recursive: true });
    fx.save();
};

// writeSog at paletteSize 65,536 (write-sog.ts:296-359; k-means.ts:137-201): N = 100,000 SH-3
// splats, 2 iterations, through the reference's own --no-gpu path (~10 min on one core).  The
// table is reproducible from its seed (makeBellSplats), so the fixture holds sha256 digests of
// the input columns, of the seven RGBA textures and of every kmeans() call's centroids and
// labels, plus meta and the draw counts -- no bulk data.
cases.sog65k = async () => {
    const fx = new Fixture('sog65k');
    const n = Number(process.env.ST_SOG65K_N || 100000), shc = 15, iters = 2, seed = 651, dseed = 652;
    const { names, cols } = makeBellSplats(n, shc, seed, 0.05);
    const table = toTable(names, cols);
    const dir = fs.mkdtempSync('/tmp/st_sog65k_');
    const metaPath = path.join(dir, 'meta.json');
    const fh = await fs.promises.open(metaPath, 'w');
    seedRandom(dseed);
    kmeansCalls.length = 0;
    recordKmeans = true;
    const t0 = Date.now();
    try {
        await quiet(() => writeSog(fh, table, metaPath, iters, 'cpu'));
    } finally {
        recordKmeans = false;
    }
    await fh.close();
    const meta = JSON.parse(fs.readFileSync(metaPath, 'utf8'));
    const files = ['means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels'];
    const tex = {};
    files.forEach((f) => {
        const t = readRGBA(path.join(dir, `${f}.webp`));
        tex[f] = { w: t.w, h: t.h, sha256: sha256(t.data) };
    });
    fx.meta = {
        generator: 'makeBellSplats', n, sh_coeffs: shc, iters, seed, draw_seed: dseed, cube_frac: 0.05,
        draws: drawCount, seconds: (Date.now() - t0) / 1000, meta,
        input_sha256: Object.fromEntries(names.map(nm => [nm, sha256(cols[nm])])),
        textures: tex,
        kmeans_calls: kmeansCalls.map(c => ({ n: c.n, d: c.d, k: c.k, iters: c.iters, draws_before: c.drawsBefore,
            draws_after: c.drawsAfter, centroids_sha256: sha256(Buffer.concat(c.centroids.map(a => Buffer.from(a.buffer)))),
            labels_sha256: sha256(c.labels) }))
    };
    // the SH palette's labels themselves (400 KB): a mismatch can then be located
    const shCall = kmeansCalls.find(c => c.d === shc * 3);
    fx.add('sh_labels', shCall.labels);
    fs.rmSync ? fs.rmSync(dir, { recursive: true }) : fs.rmdirSync(dir, { recursive: true });
    fx.save();
};

cases.filter_combine = () => {
    const fx = new Fixture('filter_combine');
    const { names, cols } = makeSplats(500, 15, 77);
    const g = new Gen(78);
    for (let i = 0; i < 40; ++i) {
        const r = g.int(500), c = names[g.int(names.length)];
        cols[c][r] = [NaN, Infinity, -Infinity][i % 3];
    }
    cols.x[0] = NaN; cols.opacity[499] = -Infinity;
    const table = toTable(names, cols);
    addTable(fx, 'in_', table);
    const out = processDataTable(table, [{ kind: 'filterNaN' }]);
    addTable(fx, 'out_', out);
    // combine (index.ts:158-210): partially overlapping schemas
    const a = new DataTable([new Column('x', new Float32Array([1, 2, 3])), new Column('y', new Float32Array([4, 5, 6])),
        new Column('tag', new Uint8Array([7, 8, 9]))]);
    const b = new DataTable([new Column('y', new Float32Array([10, 11])), new Column('z', new Float32Array([12, 13])),
        new Column('tag', new Float32Array([0.5, 1.5]))]);
    const c = new DataTable([new Column('x', new Float32Array([14])), new Column('tag', new Uint8Array([15]))]);
    [['a', a], ['b', b], ['c', c]].forEach(([nm, t]) => addTable(fx, `cmb_${nm}_`, t));
    const merged = combine([a, b, c]);
    fx.meta.cmb_out_types = merged.columns.map(col => col.dataType);
    addTable(fx, 'cmb_out_', merged);
    // by position too: the result holds two 'tag' columns (uint8 and float32)
    merged.columns.forEach((col, j) => fx.add(`cmb_out_i${j}`, col.data));

    // every column type (data-table.ts:1-27): filterNaN tests float64 columns as well, integer
    // columns are always finite; permuteRows keeps each column's type
    const tg = new Gen(79);
    const nt = 333;
    const ctors = { int8: Int8Array, uint8: Uint8Array, int16: Int16Array, uint16: Uint16Array,
        int32: Int32Array, uint32: Uint32Array, float32: Float32Array, float64: Float64Array };
    const typedCols = Object.keys(ctors).map((t) => {
        const a = new ctors[t](nt);
        for (let i = 0; i < nt; ++i) a[i] = (t.startsWith('float') ? tg.normal(0, 100) : Math.floor(tg.u() * 1e10) - 5e9);
        return new Column(`c_${t}`, a);
    });
    const f32 = typedCols[6].data, f64 = typedCols[7].data;
    [3, 50, 51, 200].forEach((r, i) => { f64[r] = [NaN, Infinity, -Infinity, NaN][i]; });
    [7, 50, 332].forEach((r, i) => { f32[r] = [Infinity, NaN, -Infinity][i]; });
    f64[9] = 1e308 * 10;  // +Infinity from arithmetic
    f64[10] = 5e-324; f64[11] = -0;
    const typed = new DataTable(typedCols);
    fx.meta.typed_types = typed.columns.map(col => col.dataType);
    addTable(fx, 'typed_in_', typed);
    const typedOut = processDataTable(typed, [{ kind: 'filterNaN' }]);
    fx.meta.typed_out_types = typedOut.columns.map(col => col.dataType);
    addTable(fx, 'typed_out_', typedOut);

    // combine over four tables: mixed types per name, a duplicate column in the first table,
    // an empty table, columns absent from some tables
    const mk = (name, ctor, vals) => new Column(name, ctor.from(vals));
    const t0 = new DataTable([mk('x', Float32Array, [1, 2]), mk('id', Uint32Array, [10, 11]), mk('x', Float32Array, [5, 6]),
        mk('w', Float64Array, [0.1, 0.2])]);
    const t1 = new DataTable([mk('id', Int32Array, [-1, -2, -3]), mk('x', Float32Array, [7, 8, 9]), mk('q', Int16Array, [300, -300, 1])]);
    const t2 = new DataTable([mk('x', Float32Array, []), mk('w', Float32Array, [])]);
    const t3 = new DataTable([mk('q', Int16Array, [4]), mk('w', Float64Array, [NaN]), mk('id', Uint32Array, [4000000000]),
        mk('b', Int8Array, [-7])]);
    const c4 = [t0, t1, t2, t3];
    c4.forEach((t, i) => {
        fx.meta[`c4_${i}_types`] = t.columns.map(col => col.dataType);
        fx.meta[`c4_${i}_names`] = t.columns.map(col => col.name);
        t.columns.forEach((col, j) => fx.add(`c4_${i}_i${j}`, col.data));
    });
    const m4 = combine(c4);
    fx.meta.c4_out_types = m4.columns.map(col => col.dataType);
    fx.meta.c4_out_names = m4.columns.map(col => col.name);
    m4.columns.forEach((col, j) => fx.add(`c4_out_i${j}`, col.data));
    fx.save();
};

// processDataTable over every action kind (process.ts:64-145) followed by writeCompressedPly
// (write-compressed-ply.ts:31-115): the CLI's `in.ply [actions] out.compressed.ply`
// (index.ts:463-496).  Per case: the input table, the processed table (names, types, data) and
// the four file writes of the compressed PLY (or the error either step threw).
cases.process_chain = async () => {
    const fx = new Fixture('process_chain');
    const V = (x, y, z) => new pc.Vec3(x, y, z);
    const specs = [];
    {   // BASELINE config 3: -r 0,45,0 --filterNaN
        const { names, cols } = makeSplats(3000, 15, 901, { cubeFrac: 0.1 });
        const g = new Gen(902);
        for (let i = 0; i < 30; ++i) cols[names[g.int(names.length)]][g.int(3000)] = [NaN, Infinity, -Infinity][i % 3];
        specs.push(['config3', names, cols, [{ kind: 'rotate', value: V(0, 45, 0) }, { kind: 'filterNaN' }]]);
    }
    {   // filterByValue / scale / filterBands(1) with NaN in the filtered column
        const { names, cols } = makeSplats(2500, 15, 903, { cubeFrac: 0.05 });
        cols.opacity[3] = NaN; cols.opacity[4] = 0.5; cols.opacity[5] = -0;
        specs.push(['value_bands1', names, cols, [{ kind: 'filterByValue', columnName: 'opacity', comparator: 'gt', value: 0.5 },
            { kind: 'scale', value: 2 }, { kind: 'filterBands', value: 1 }]]);
    }
    {   // filterBands(2), lte, translate, filterNaN, then a param (no-op)
        const { names, cols } = makeSplats(2000, 15, 904);
        cols.x[7] = 0; cols.x[8] = -0; cols.y[9] = NaN;
        specs.push(['bands2_lte', names, cols, [{ kind: 'filterBands', value: 2 },
            { kind: 'filterByValue', columnName: 'x', comparator: 'lte', value: 0 },
            { kind: 'translate', value: V(1, 2, 3) }, { kind: 'filterNaN' }, { kind: 'param', name: 'a', value: 'b' }]]);
    }
    {   // eq / neq on exact values, a missing column (neq keeps all, eq keeps none is a separate case),
        // an unknown comparator (keeps all), gte / lt
        const { names, cols } = makeSplats(1500, 3, 905, { cubeFrac: 0.2 });
        for (let i = 0; i < 1500; i += 7) cols.scale_0[i] = -4;
        cols.scale_0[11] = NaN;
        specs.push(['eq_neq', names, cols, [{ kind: 'filterByValue', columnName: 'scale_0', comparator: 'neq', value: -4 },
            { kind: 'filterByValue', columnName: 'nope', comparator: 'neq', value: 1 },
            { kind: 'filterByValue', columnName: 'z', comparator: 'bogus', value: 1 },
            { kind: 'filterByValue', columnName: 'y', comparator: 'gte', value: -5 },
            { kind: 'filterByValue', columnName: 'rot_0', comparator: 'lt', value: 1.25 },
            { kind: 'rotate', value: V(-30.5, 170, 45.25) }]]);
    }
    {   // eq keeps the exact matches only; SH1 -> bands 0
        const { names, cols } = makeSplats(1200, 3, 906);
        for (let i = 0; i < 1200; i += 5) cols.f_dc_1[i] = 0.25;
        specs.push(['eq_bands0', names, cols, [{ kind: 'filterByValue', columnName: 'f_dc_1', comparator: 'eq', value: 0.25 },
            { kind: 'filterBands', value: 0 }, { kind: 'rotate', value: V(90, 0, 0) }]]);
    }
    {   // every row filtered out
        const { names, cols } = makeSplats(700, 8, 907);
        specs.push(['empty', names, cols, [{ kind: 'filterByValue', columnName: 'x', comparator: 'gt', value: 1e30 }]]);
    }
    {   // SH0 table, filterBands above its band (no-op), two filters in a row
        const { names, cols } = makeSplats(900, 0, 908);
        cols.opacity[1] = Infinity;
        specs.push(['sh0_two_filters', names, cols, [{ kind: 'filterBands', value: 3 }, { kind: 'filterNaN' },
            { kind: 'filterByValue', columnName: 'opacity', comparator: 'lt', value: 2 }, { kind: 'scale', value: 0.5 }]]);
    }
    {   // transforms after a filterBands (before any filter) rotate the renamed band-1 view, whose
        // columns are the input's arrays (process.ts:110-134): the input is mutated through them
        const { names, cols } = makeSplats(1800, 15, 909);
        cols.z[5] = NaN;
        specs.push(['bands_rotate_nan', names, cols, [{ kind: 'filterBands', value: 1 },
            { kind: 'rotate', value: V(10, 20, 30) }, { kind: 'translate', value: V(1, 0, 0) }, { kind: 'filterNaN' }]]);
    }
    {   // transforms only: the result IS the input table, mutated
        const { names, cols } = makeSplats(1000, 8, 910);
        specs.push(['transforms_only', names, cols, [{ kind: 'scale', value: 1.5 }, { kind: 'rotate', value: V(0, 0, 90) }]]);
    }
    fx.meta.cases = specs.map(s => s[0]);
    const actionsMeta = (acts) => acts.map(a => (a.value && a.value.x !== undefined)
        ? Object.assign({}, a, { value: [a.value.x, a.value.y, a.value.z] }) : a);
    for (const [name, names, cols, acts] of specs) {
        const table = toTable(names, cols);
        fx.meta[`${name}_actions`] = actionsMeta(acts);
        addTable(fx, `${name}_in_`, table);
        const out = processDataTable(table, acts);
        fx.meta[`${name}_out_types`] = out.columns.map(c => c.dataType);
        addTable(fx, `${name}_out_`, out);
        // the input table afterwards: the transforms before the first filter mutate it in place
        addTable(fx, `${name}_after_`, table);
        const { writes, handle } = captureHandle();
        try {
            await quiet(() => writeCompressedPly(handle, out));
            const u8 = (b) => new Uint8Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.length));
            fx.add(`${name}_header`, u8(writes[0]));
            fx.add(`${name}_chunk`, new Float32Array(u8(writes[1]).buffer));
            fx.add(`${name}_vertex`, new Uint32Array(u8(writes[2]).buffer));
            fx.add(`${name}_sh`, u8(writes[3]));
        } catch (e) {
            fx.meta[`${name}_write_error`] = String(e);
        }
    }
    fx.save();
};

(async () => {
    for (const name of Object.keys(cases)) {
        if (only.length && only.indexOf(name) < 0) continue;
        process.stderr.write(`case ${name}\n`);
        await cases[name]();
    }
})().catch((e) => { console.error(e); process.exit(1); });
