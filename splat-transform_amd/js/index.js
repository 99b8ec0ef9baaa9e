'use strict';
// splat-hip host module: the reference's hot-path functions, same names,
// argument meaning and in-place mutation, executed on MI355X through the N-API
// addon (../napi/addon.c) over the C-ABI (include/st_abi.h).  Plain JS for
// Node >= 12 (no `??`, no `?.`).  A DataTable is anything shaped like the
// reference's (src/data-table.ts:5-150): {columns: [{name, data}], numRows,
// getColumnByName(name), hasColumn(name)}; the Column/DataTable classes below
// are a minimal stand-in for standalone use.
//
//   transform(dataTable, t, r, s)           transform.ts:12-65
//   generateOrdering(dataTable, indices)    ordering.ts:4-110
//   filterNaN(dataTable)                    process.ts:84-95 (+ filter :47-61, permuteRows)
//   combine(dataTables)                     index.ts:158-210
//   packCompressed(dataTable)               write-compressed-ply.ts:56-109 (the chunk loop)
//   processDataTable(dataTable, actions)    process.ts:64-145 (one upload for the whole list)
//   writeCompressedPly(fh, dataTable[, actions])  write-compressed-ply.ts:31-115 (actions first,
//                                           same device call: the CLI's config-3 path; a real
//                                           FileHandle is written as the arrays leave HBM)
//   compressPlyFile(inFh, outFh, actions)   readPly + processDataTable + writeCompressedPly, the rows
//   sogFromPlyFile(inFh, actions, iters)    resident in HBM (the CLI's one-input paths, index.ts:463-496)
//   kmeans(points, k, iterations)           k-means.ts:137-201 (--no-gpu results)
//   cluster1d(dataTable, iterations)        write-sog.ts:56-99
//   sogTextures(dataTable, iterations)      write-sog.ts:110-370 (textures + meta, before WebP/ZIP)
//   writeSogBundle(dataTable, iterations[, actions])  write-sog.ts:110-370 to a .sog (WebP + CRC + ZIP on
//                                           the device; actions first, same device call)
//   WebpEncoder                             utils/webp.ts:19-41 (encodeLosslessRGBA)
//   readPly(fileHandle)                     readers/read-ply.ts:111-191
//   isCompressedPly / decompressPly(ply)    readers/decompress-ply.ts:6-232
//
// Math.random: the device consumes the reference's draws in the reference's
// order.  Draws are taken from Math.random up front; the ones a call did not
// consume are kept in `pending` and served first to the next call, so the
// process-wide stream is exactly what the reference would have consumed.

const path = require('path');

const addon = require(path.join(__dirname, '..', 'napi', 'build', 'addon.node'));

class Column {
    constructor(name, data) {
        this.name = name;
        this.data = data;
    }
}

// A readPly column whose values are still only in HBM (the addon's resident read): its memory is
// allocated but unfilled, and `data` copies the values down on first access (addon.materialize),
// after which it is an ordinary own property.  Until then nothing in JS holds the array, so it is
// unchanged by construction and writeSogFile runs on the device copy (st_sog_file: no upload, no
// compare).  Assigning `data` drops the resident copy.
const kResident = Symbol('splat-hip resident column');
const residentColumn = (name, ta) => {
    const c = new Column(name, ta);
    const settle = (v) => {
        delete c[kResident];
        Object.defineProperty(c, 'data', { value: v, writable: true, enumerable: true, configurable: true });
    };
    c[kResident] = ta;
    Object.defineProperty(c, 'data', {
        enumerable: true,
        configurable: true,
        get() {
            addon.materialize(ta);
            settle(ta);
            return ta;
        },
        set(v) { settle(v); }
    });
    return c;
};
// the column's array without copying a resident one down (only for writeSogFile, which reads
// resident columns on the device; every other host form would copy them down anyway)
const deviceOrHost = c => (c[kResident] !== undefined ? c[kResident] : c.data);
const rowsOf = c => deviceOrHost(c).length;

class DataTable {
    constructor(columns) {
        if (columns.length === 0) throw new Error('DataTable must have at least one column');
        for (let i = 1; i < columns.length; ++i) {
            if (rowsOf(columns[i]) !== rowsOf(columns[0])) {
                throw new Error(`Column ${columns[i].name} has a different number of rows`);
            }
        }
        this.columns = columns;
    }
    get numRows() { return rowsOf(this.columns[0]); }
    get numColumns() { return this.columns.length; }
    getColumn(i) { return this.columns[i]; }
    getColumnByName(name) { return this.columns.find(c => c.name === name); }
    hasColumn(name) { return this.columns.some(c => c.name === name); }
    getColumnNames() { return this.columns.map(c => c.name); }
}

// ---- Math.random stream --------------------------------------------------------
// draws taken from Math.random but not consumed yet, oldest first (a typed array: a call hands
// back ~10^6 unconsumed draws, copied as memory rather than element by element)
let pending = new Float64Array(0);

const takeDraws = (count) => {
    const out = new Float64Array(count);
    const m = Math.min(count, pending.length);
    out.set(pending.subarray(0, m));
    for (let i = m; i < count; ++i) out[i] = Math.random();
    pending = pending.subarray(m);
    return out;
};

const giveBack = (draws, used) => {
    const back = draws.subarray(used);
    const merged = new Float64Array(back.length + pending.length);
    merged.set(back);
    merged.set(pending, back.length);
    pending = merged;
};

// drop the draws taken from Math.random but not consumed yet (call after re-seeding Math.random:
// the next call then starts on the new stream)
const resetRandomStream = () => { pending = new Float64Array(0); };

// error.code of a call that ran out of draws (ST_ERR_DRAWS = -4, st_abi.h; the addon's throw_st)
const ST_ERR_DRAWS_CODE = 'ST_STATUS_4';

// run fn(draws) with enough draws; a short buffer (ST_ERR_DRAWS) is retried with
// a longer one that starts with the same values, so the stream is unchanged
const withDraws = (estimate, fn) => {
    let count = Math.max(estimate, 64);
    for (;;) {
        const draws = takeDraws(count);
        try {
            const res = fn(draws);
            giveBack(draws, res.used);
            return res;
        } catch (e) {
            giveBack(draws, 0);
            if (e.code !== ST_ERR_DRAWS_CODE) throw e;
            count *= 2;
        }
    }
};

// ---- helpers ---------------------------------------------------------------------
const f32Columns = (dataTable) => {
    const cols = [];
    const names = [];
    for (const c of dataTable.columns) {
        if (!(c.data instanceof Float32Array)) continue;
        cols.push(c.data);
        names.push(c.name);
    }
    return { cols, names };
};

const shCoeffsOf = (dataTable) => {
    // band detection rule of transform.ts:20 / write-compressed-ply.ts:32
    const idx = [9, 24, -1];
    const miss = (() => {
        for (let i = 0; i < 45; ++i) if (!dataTable.hasColumn(`f_rest_${i}`)) return i;
        return -1;
    })();
    const band = idx.indexOf(miss) + 1;
    return [0, 3, 8, 15][band];
};

// ---- the path ------------------------------------------------------------------------
// the columns transform.ts:16-20 reads and writes (position, rotation, scale, SH by the band rule)
const transformColumns = (dataTable) => {
    const groups = [['x', 'y', 'z'], ['rot_0', 'rot_1', 'rot_2', 'rot_3'], ['scale_0', 'scale_1', 'scale_2']];
    const names = [];
    groups.forEach((g) => { if (g.every(n => dataTable.hasColumn(n))) names.push(...g); });
    for (let i = 0; i < 3 * shCoeffsOf(dataTable); ++i) names.push(`f_rest_${i}`);
    return names;
};

// t: {x, y, z} (Vec3), r: {x, y, z, w} (Quat), s: number -- mutates the columns in place.
// The device path computes in f64 on the columns' numbers and stores as the TypedArray does
// (float32 tables: float32 stores; other types through st_transform_t, as getRow / setRow).
const transform = (dataTable, t, r, s) => {
    const typed = transformColumns(dataTable).some(n => !(dataTable.getColumnByName(n).data instanceof Float32Array));
    if (typed) {
        addon.transformTyped(dataTable.columns.map(c => c.data), dataTable.columns.map(c => c.name),
            [t.x, t.y, t.z], [r.x, r.y, r.z, r.w], s);
        return;
    }
    const { cols, names } = f32Columns(dataTable);
    addon.transform(cols, names, [t.x, t.y, t.z], [r.x, r.y, r.z, r.w], s);
};

const quatFromEuler = (x, y, z) => {
    const q = addon.quatFromEuler(x, y, z);
    return { x: q[0], y: q[1], z: q[2], w: q[3] };
};

const generateOrdering = (dataTable, indices) => {
    const x = dataTable.getColumnByName('x').data;
    const y = dataTable.getColumnByName('y').data;
    const z = dataTable.getColumnByName('z').data;
    // ordering.ts:32-47 reads the numbers of any column type
    if (!(x instanceof Float32Array && y instanceof Float32Array && z instanceof Float32Array)) {
        return addon.mortonOrderTyped(x, y, z, indices);
    }
    return addon.mortonOrder(x, y, z, indices);
};

// rows whose every column value isFinite, in order (filterNaN): every column type, the
// compaction and the row gather on the device, each column keeping its type
const filterNaN = (dataTable) => {
    const out = addon.filterNaN(dataTable.columns.map(c => c.data));
    return new DataTable(dataTable.columns.map((c, i) => new Column(c.name, out[i])));
};

const PLY_TYPE = { Int8Array: 1, Uint8Array: 2, Int16Array: 3, Uint16Array: 4, Int32Array: 5, Uint32Array: 6,
    Float32Array: 7, Float64Array: 8 };

// index.ts:158-210: columns united by (name, dataType), rows appended, absent columns zero
const combine = (dataTables) => {
    if (dataTables.length === 1) return dataTables[0];
    const layout = addon.combineLayout(dataTables.map(t => ({
        names: t.columns.map(c => c.name), types: t.columns.map(c => PLY_TYPE[c.data.constructor.name] || 0)
    })));
    const total = dataTables.reduce((sum, t) => sum + t.numRows, 0);
    const result = layout.map(([t, j]) => {
        const c = dataTables[t].columns[j];
        return new Column(c.name, new c.data.constructor(total));
    });
    const target = (c) => result.find(r => r.name === c.name && r.data.constructor === c.data.constructor);
    let offset = 0;
    for (const t of dataTables) {
        for (const c of t.columns) target(c).data.set(c.data, offset);
        offset += t.numRows;
    }
    return new DataTable(result);
};

// the chunk / vertex / sh arrays writeCompressedPly writes after its header
const packCompressed = (dataTable) => {
    if (dataTable.columns.some(c => !(c.data instanceof Float32Array))) {
        // any column type: the writer's device path over the typed table (no actions)
        const res = addon.compressedPly(dataTable.columns.map(c => c.data), dataTable.columns.map(c => c.name), []);
        return { chunk: res.chunk, vertex: res.vertex, sh: res.sh };
    }
    const n = dataTable.numRows;
    const order = new Uint32Array(n);
    for (let i = 0; i < n; ++i) order[i] = i;
    generateOrdering(dataTable, order);
    const { cols, names } = f32Columns(dataTable);
    return addon.packCompressed(cols, names, order, 3 * shCoeffsOf(dataTable));
};

// ---- processDataTable / writeCompressedPly (process.ts:64-145, write-compressed-ply.ts:31-115) ----
// ProcessAction objects as the reference's CLI builds them (process.ts:6-42): Vec3 values for
// translate / rotate, a number for scale, {columnName, comparator, value} for filterByValue.
// Normalised for the addon: k = st_action_kind, transform params as t / r / s.
const ACTION = { transform: 1, filterNaN: 2, filterByValue: 3, filterBands: 4, param: 5 };
const COMPARE = { lt: 0, lte: 1, gt: 2, gte: 3, eq: 4, neq: 5 };
const normaliseActions = actions => actions.map((a) => {
    switch (a.kind) {
        case 'translate':
            return { k: ACTION.transform, t: [a.value.x, a.value.y, a.value.z], r: [0, 0, 0, 1], s: 1 };
        case 'rotate': {
            const q = addon.quatFromEuler(a.value.x, a.value.y, a.value.z);
            return { k: ACTION.transform, t: [0, 0, 0], r: q, s: 1 };
        }
        case 'scale':
            return { k: ACTION.transform, t: [0, 0, 0], r: [0, 0, 0, 1], s: a.value };
        case 'filterNaN':
            return { k: ACTION.filterNaN };
        case 'filterByValue':
            return { k: ACTION.filterByValue, column: String(a.columnName),
                compare: Object.prototype.hasOwnProperty.call(COMPARE, a.comparator) ? COMPARE[a.comparator] : -1,
                value: Number(a.value) };
        case 'filterBands':
            return { k: ACTION.filterBands, bands: a.value };
        case 'param':
            return { k: ACTION.param };
        default:
            return { k: 0 };  // unknown kinds: the reference's switch ignores them
    }
}).filter(a => a.k !== 0);

// the columns processDataTable leaves: filterBands renames / drops f_rest columns against the
// ORIGINAL table's band (process.ts:110-134); [name, index of the source column]
const processSchema = (dataTable, actions) => {
    const inCoeffs = shCoeffsOf(dataTable);
    let cols = dataTable.columns.map((c, i) => [c.name, i]);
    for (const a of actions) {
        if (a.kind !== 'filterBands') continue;
        const outCoeffs = [0, 3, 8, 15][a.value];
        if (!(outCoeffs < inCoeffs)) continue;
        const map = {};
        for (let i = 0; i < inCoeffs; ++i) {
            for (let j = 0; j < 3; ++j) map[`f_rest_${i + j * inCoeffs}`] = i < outCoeffs ? `f_rest_${i + j * outCoeffs}` : null;
        }
        cols = cols.map(([n, i]) => (Object.prototype.hasOwnProperty.call(map, n) ? [map[n], i] : [n, i]))
            .filter(([n]) => n !== null);
    }
    return cols;
};

// processDataTable(dataTable, processActions) -> DataTable: the whole action list on the device
// with one upload and one download (transform passes, filters and the row gathers in HBM).
// As in the reference, the transforms before the first filter mutate the caller's columns
// (process.ts:65-83: `result` is the input table until a filter copies it; filterBands only
// renames, its columns keep the input's arrays): those run first and are written back into the
// input arrays, the rest runs on the mutated table.
const isTransform = a => a.kind === 'translate' || a.kind === 'rotate' || a.kind === 'scale';
const isFilter = a => a.kind === 'filterNaN' || a.kind === 'filterByValue';
const processDataTable = (dataTable, processActions) => {
    const cols = () => dataTable.columns.map(c => c.data);
    const names = dataTable.columns.map(c => c.name);
    let first = processActions.findIndex(isFilter);
    if (first < 0) first = processActions.length;
    const region = processActions.slice(0, first);
    const rs = processSchema(dataTable, region);
    if (region.some(isTransform)) {
        const out = addon.process(cols(), names, normaliseActions(region), rs.map(s => s[0]), rs.map(s => s[1]));
        rs.forEach((s, j) => dataTable.columns[s[1]].data.set(out[j]));
    }
    if (first === processActions.length) {
        // no filter: the result shares the input's (mutated) arrays, renamed by filterBands
        return rs.length === dataTable.columns.length && rs.every((s, j) => s[1] === j && s[0] === names[j]) ?
            dataTable : new DataTable(rs.map(s => new Column(s[0], dataTable.columns[s[1]].data)));
    }
    const rest = processActions.filter((a, i) => i >= first || !isTransform(a));  // filterBands re-applied
    const schema = processSchema(dataTable, rest);
    const out = addon.process(cols(), names, normaliseActions(rest), schema.map(s => s[0]), schema.map(s => s[1]));
    return new DataTable(schema.map((s, j) => new Column(s[0], out[j])));
};

const CHUNK_PROPS_OUT = ['min_x', 'min_y', 'min_z', 'max_x', 'max_y', 'max_z', 'min_scale_x', 'min_scale_y',
    'min_scale_z', 'max_scale_x', 'max_scale_y', 'max_scale_z', 'min_r', 'min_g', 'min_b', 'max_r', 'max_g', 'max_b'];
const VERTEX_PROPS_OUT = ['packed_position', 'packed_rotation', 'packed_scale', 'packed_color'];

// write-compressed-ply.ts:31-115: header + chunk + vertex + sh writes.  With processActions the
// actions run first in the same device call (the CLI's `in.ply [actions] out.compressed.ply`:
// the table crosses PCIe once each way).  version: the package version of the header comment.
// A real fs.promises FileHandle (a numeric fd) takes the streamed form: the library writes the
// header and the arrays at the handle's position as they leave HBM (st_compressed_ply_file) and
// leaves the position after them; any other handle gets the reference's four write() calls.
const hasFd = h => h && typeof h.fd === 'number' && h.fd >= 0;
const writeCompressedPly = async (fileHandle, dataTable, processActions, version) => {
    if (hasFd(fileHandle)) {
        addon.compressedPlyTableToFile(dataTable.columns.map(c => c.data), dataTable.columns.map(c => c.name),
            normaliseActions(processActions || []), fileHandle.fd, version || '0.10.1');
        return;
    }
    const res = addon.compressedPly(dataTable.columns.map(c => c.data), dataTable.columns.map(c => c.name),
        normaliseActions(processActions || []));
    await fileHandle.write(Buffer.from(compressedPlyHeader(res.numRows, res.shCoeffs, version), 'utf8'));
    await fileHandle.write(new Uint8Array(res.chunk.buffer));
    await fileHandle.write(new Uint8Array(res.vertex.buffer));
    await fileHandle.write(res.sh);
};

// the CLI's one-input paths straight from the file (index.ts:463-496): readPly + processDataTable +
// the writer in one device call, the rows resident in HBM (read page cache -> pinned -> HBM); only
// the outputs cross back.  inHandle / outHandle: fs.promises FileHandles.
const compressedPlyHeader = (numSplats, outputSHCoeffs, version) => {
    const shHeader = outputSHCoeffs ? [`element sh ${numSplats}`].concat(
        new Array(outputSHCoeffs * 3).fill('').map((_, i) => `property uchar f_rest_${i}`)) : [];
    return [].concat(
        'ply', 'format binary_little_endian 1.0', `comment Generated by splat-transform ${version || '0.10.1'}`,
        `element chunk ${Math.ceil(numSplats / 256)}`, CHUNK_PROPS_OUT.map(p => `property float ${p}`),
        `element vertex ${numSplats}`, VERTEX_PROPS_OUT.map(p => `property uint ${p}`),
        shHeader, 'end_header\n').join('\n');
};

const compressPlyFile = async (inHandle, outHandle, processActions, version) => {
    if (hasFd(outHandle)) {  // streamed into the file as the arrays leave HBM (st_ply_compressed_ply_file)
        addon.compressedPlyToFile(inHandle.fd, normaliseActions(processActions || []), outHandle.fd,
            version || '0.10.1');
        return;
    }
    const res = addon.compressedPlyFromFile(inHandle.fd, normaliseActions(processActions || []));
    await outHandle.write(Buffer.from(compressedPlyHeader(res.numRows, res.shCoeffs, version), 'utf8'));
    await outHandle.write(new Uint8Array(res.chunk.buffer));
    await outHandle.write(new Uint8Array(res.vertex.buffer));
    await outHandle.write(res.sh);
};

const sogFromPlyFile = (inHandle, processActions, iterations) => {
    const k = 65536;
    const date = new Date();
    const dosTime = (date.getHours() << 11) | (date.getMinutes() << 5) | Math.floor(date.getSeconds() / 2);
    const dosDate = ((date.getFullYear() - 1980) << 9) | ((date.getMonth() + 1) << 5) | date.getDate();
    const acts = normaliseActions(processActions || []);
    const res = withDraws(4 * 256 * (iterations + 1) + k * (iterations + 1) + 4096,
        draws => addon.sogBundleFromFile(inHandle.fd, acts, iterations, draws, dosTime, dosDate));
    return Promise.resolve(res.archive);
};

const kmeans = (points, k, iterations) => {
    const cols = points.columns.map(c => c.data);
    const n = points.numRows;
    const res = withDraws(k * (iterations + 1) + 1024, draws => addon.kmeans(cols, k, iterations, draws));
    const kk = Math.min(k, n);
    const centroids = new DataTable(points.columns.map((c, i) =>
        new Column(c.name, res.centroids.slice(i * kk, (i + 1) * kk))));
    return Promise.resolve({ centroids, labels: res.labels });
};

const cluster1d = (dataTable, iterations) => {
    const cols = dataTable.columns.map(c => c.data);
    const n = dataTable.numRows;
    const res = withDraws(256 * (iterations + 1) + 64, draws => addon.cluster1d(cols, iterations, draws));
    const labels = new DataTable(dataTable.columns.map((c, i) =>
        new Column(c.name, res.labels.slice(i * n, (i + 1) * n))));
    const centroids = new DataTable([new Column('data', res.centroids)]);
    return Promise.resolve({ centroids, labels });
};

// writeSog's device work: the seven RGBA textures and the meta.json fields (columns of any type:
// write-sog.ts reads positions, rotations and opacity as numbers, cluster1d and the k-means
// points through Float32Arrays)
const sogTextures = (dataTable, iterations) => {
    const k = 65536;
    return Promise.resolve(withDraws(4 * 256 * (iterations + 1) + k * (iterations + 1) + 4096,
        draws => addon.sogProcess(dataTable.columns.map(c => c.data), dataTable.columns.map(c => c.name), [],
            iterations, draws)));
};

// utils/webp.ts:19-41: same class shape; the stream is a valid lossless WebP of the same
// pixels (encoded on the device), not libwebp's bytes
class WebpEncoder {
    static async create() { return new WebpEncoder(); }

    encodeLosslessRGBA(rgba, width, height, stride = width * 4) {
        return addon.webpLossless(rgba, width, height, stride);
    }
}

// writeSog to a .sog bundle (write-sog.ts:110-370 with its ZipWriter): the archive bytes.
// The ZIP clock is taken like zip-writer.ts:39-41 when the archive is written.
const writeSogBundle = (dataTable, iterations, processActions) => {
    const k = 65536;
    const date = new Date();
    const dosTime = (date.getHours() << 11) | (date.getMinutes() << 5) | Math.floor(date.getSeconds() / 2);
    const dosDate = ((date.getFullYear() - 1980) << 9) | ((date.getMonth() + 1) << 5) | date.getDate();
    const acts = normaliseActions(processActions || []);
    // no actions and float32 columns only: st_sog_bundle, which reads readPly's untouched columns
    // where they are in HBM (deviceOrHost: nothing copied down); otherwise the typed chain
    const plain = acts.length === 0 && dataTable.columns.every(c => deviceOrHost(c) instanceof Float32Array);
    const res = withDraws(4 * 256 * (iterations + 1) + k * (iterations + 1) + 4096,
        draws => (plain ? addon.sogBundle(dataTable.columns.map(deviceOrHost), dataTable.columns.map(c => c.name),
            iterations, draws, dosTime, dosDate) :
            addon.sogBundleProcess(dataTable.columns.map(c => c.data), dataTable.columns.map(c => c.name), acts,
                iterations, draws, dosTime, dosDate)));
    return Promise.resolve(res.archive);
};

// writeSog into an open FileHandle (write-sog.ts:110-370 and the CLI's write of the .sog): the
// archive is streamed into the file while the SH palette k-means runs (st_sog_file); the file
// holds writeSogBundle's bytes and is cut to their length.  The handle must be a seekable file
// (the archive is written at absolute offsets): a pipe's handle throws before any work.  Float32
// columns; readPly's columns that JS has not read are taken from HBM where they are.
const writeSogFile = (fileHandle, dataTable, iterations) => {
    const k = 65536;
    const date = new Date();
    const dosTime = (date.getHours() << 11) | (date.getMinutes() << 5) | Math.floor(date.getSeconds() / 2);
    const dosDate = ((date.getFullYear() - 1980) << 9) | ((date.getMonth() + 1) << 5) | date.getDate();
    const res = withDraws(4 * 256 * (iterations + 1) + k * (iterations + 1) + 4096,
        draws => addon.sogFile(fileHandle.fd, dataTable.columns.map(deviceOrHost), dataTable.columns.map(c => c.name),
            iterations, draws, dosTime, dosDate));
    return Promise.resolve(res.size);
};

// readers/read-ply.ts:111-191: {comments, elements: [{name, dataTable}]} from an open FileHandle
// (rows stream through pinned memory into HBM and are transposed to columns there; the columns
// stay there until JS first reads a column's `data` -- residentColumn above)
const readPly = (fileHandle) => {
    const r = addon.readPly(fileHandle.fd);
    return Promise.resolve({
        comments: r.comments,
        elements: r.elements.map(e => ({
            name: e.name,
            dataTable: new DataTable(e.columns.map(c => (c.lazy ? residentColumn(c.name, c.data) :
                new Column(c.name, c.data))))
        }))
    });
};

const CHUNK_PROPS = ['min_x', 'min_y', 'min_z', 'max_x', 'max_y', 'max_z', 'min_scale_x', 'min_scale_y',
    'min_scale_z', 'max_scale_x', 'max_scale_y', 'max_scale_z', 'min_r', 'min_g', 'min_b', 'max_r', 'max_g', 'max_b'];
const VERTEX_PROPS = ['packed_position', 'packed_rotation', 'packed_scale', 'packed_color'];

// readers/decompress-ply.ts:6-80 (schema check, host)
const isCompressedPly = (ply) => {
    const has = (dt, names, ctor) => names.every((n) => {
        const c = dt.getColumnByName(n);
        return c && c.data instanceof ctor;
    });
    const ne = ply.elements.length;
    if (ne !== 2 && ne !== 3) return false;
    const chunk = ply.elements.find(e => e.name === 'chunk');
    if (!chunk || !has(chunk.dataTable, CHUNK_PROPS, Float32Array)) return false;
    const vertex = ply.elements.find(e => e.name === 'vertex');
    if (!vertex || !has(vertex.dataTable, VERTEX_PROPS, Uint32Array)) return false;
    if (Math.ceil(vertex.dataTable.numRows / 256) !== chunk.dataTable.numRows) return false;
    if (ne === 3) {
        const sh = ply.elements.find(e => e.name === 'sh');
        if (!sh) return false;
        const d = sh.dataTable;
        if ([9, 24, 45].indexOf(d.numColumns) === -1) return false;
        for (let i = 0; i < d.numColumns; ++i) {
            const c = d.getColumnByName(`f_rest_${i}`);
            if (!c || !(c.data instanceof Uint8Array)) return false;
        }
        if (d.numRows !== vertex.dataTable.numRows) return false;
    }
    return true;
};

// readers/decompress-ply.ts:82-232 (decoded on the device)
const decompressPly = (ply) => {
    const chunk = ply.elements.find(e => e.name === 'chunk').dataTable;
    const vertex = ply.elements.find(e => e.name === 'vertex').dataTable;
    const shEl = ply.elements.find(e => e.name === 'sh');
    const shCols = shEl ? shEl.dataTable.columns : [];
    const out = addon.decompressPly(CHUNK_PROPS.map(n => chunk.getColumnByName(n).data),
        VERTEX_PROPS.map(n => vertex.getColumnByName(n).data), shCols.map(c => c.data));
    const names = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity', 'rot_0', 'rot_1', 'rot_2', 'rot_3',
        'scale_0', 'scale_1', 'scale_2'].concat(shCols.map(c => c.name));
    return new DataTable(out.map((d, i) => new Column(names[i], d)));
};

// the GPUs writeSog shards its rows over (st_set_devices; the reference's device choice is
// write-sog.ts:241-243): 1 (default) = one device
const setDevices = (n) => addon.setDevices(n);
const getDevices = () => addon.getDevices();
// {version, path} of the RCCL the library's collectives run on (the same file under every host)
const rcclInfo = () => addon.rcclInfo();

module.exports = {
    resetRandomStream,
    setDevices,
    getDevices,
    rcclInfo,
    Column,
    DataTable,
    addon,
    transform,
    quatFromEuler,
    generateOrdering,
    filterNaN,
    combine,
    packCompressed,
    processDataTable,
    writeCompressedPly,
    compressPlyFile,
    sogFromPlyFile,
    kmeans,
    cluster1d,
    sogTextures,
    WebpEncoder,
    writeSogBundle,
    writeSogFile,
    readPly,
    isCompressedPly,
    decompressPly
};
