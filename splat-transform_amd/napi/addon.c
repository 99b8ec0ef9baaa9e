/*
 * addon.c -- N-API (v8, Node >= 12) binding of libsplat_hip.so for the
 * reference's Node host.  Thin: it borrows the TypedArray storage of the
 * caller's DataTable columns for the duration of one call (no copies on the
 * JS side), forwards to the C-ABI in include/st_abi.h and turns a negative
 * st_status into a thrown JS Error carrying st_last_error().
 *
 * Exports (js/index.js wraps them in the reference's signatures):
 *   version() -> number                       st_abi_version
 *   deviceCount() -> number                   st_device_count
 *   rcclInfo() -> {version, path}             st_rccl_info (the RCCL the collectives run on)
 *   lastHostReuse() -> {columns, bytes}       st_ctx_last_host_reuse (readPly's resident columns)
 *   transform(cols, names, t[3], r[4], s)     st_transform_params_make + st_transform
 *                                             (transform.ts:12-65)
 *   quatFromEuler(ex, ey, ez) -> [x,y,z,w]    Quat.setFromEulerAngles (process.ts:75-79)
 *   filterFinite(cols) -> Uint32Array         filterNaN's row predicate (process.ts:84-95)
 *   mortonOrder(x, y, z, indices)             generateOrdering (ordering.ts:4-110), in place
 *   packCompressed(cols, names, order, nsh)   writeCompressedPly chunk loop
 *        -> {chunk, vertex, sh}               (write-compressed-ply.ts:56-109)
 *   kmeans(cols, k, iters, draws)             kmeans --no-gpu (k-means.ts:137-201)
 *        -> {centroids, labels, used}
 *   cluster1d(cols, iters, draws)             cluster1d (write-sog.ts:56-99)
 *        -> {centroids, labels, used}
 *   sog(cols, names, iters, draws)            writeSog textures + meta (write-sog.ts:110-370)
 *        -> {meta fields, textures, used}
 *   webpLossless(rgba, w, h, stride) -> Buffer WebpEncoder.encodeLosslessRGBA (utils/webp.ts:19-41,
 *                                             lib/webp_encode.c:19-29)
 *   sogBundle(cols, names, iters, draws, dosTime, dosDate)
 *   sogFile(fd, cols, names, iters,        writeSog into an open file (st_sog_file): the .sog streamed
 *           draws, dosTime, dosDate)        while the SH k-means runs; {used, size}
 *        -> {archive: Buffer, used}           writeSog to a .sog (write-sog.ts:110-370 +
 *                                             serialize/zip-writer.ts)
 *   readPly(fd) -> {comments, elements:       readPly (readers/read-ply.ts:111-191); the values
 *        [{name, columns: [{name, data,       stay in HBM (st_ply_read_resident) and `data` is
 *          lazy}]}]}                          unfilled while `lazy` (ST_READ_RESIDENT=0: filled)
 *   materialize(typedArray)                   a lazy column's values copied down (st_ply_materialize)
 *   decompressPly(chunk[18], vertex[4], sh[]) decompressPly (readers/decompress-ply.ts:82-232)
 *        -> Float32Array[14 + sh.length]
 *   compressedPly(cols, names, actions)       processDataTable + writeCompressedPly's arrays, one
 *        -> {numRows, shCoeffs, chunk,        upload (process.ts:64-145, write-compressed-ply.ts:
 *            vertex, sh}                      31-115)
 *   process(cols, names, actions, outNames,   processDataTable, one upload (process.ts:64-145)
 *           outSrc) -> TypedArray[]
 *   compressedPlyFromFile(fd, actions)        readPly + processDataTable + writeCompressedPly's
 *        -> {numRows, shCoeffs, chunk,        arrays, the rows resident in HBM (index.ts:463-496)
 *            vertex, sh}
 *   compressedPlyToFile(inFd, actions,        readPly + processDataTable + writeCompressedPly into
 *        outFd, version) -> {numRows,         outFd, written as the arrays leave HBM
 *        shCoeffs, size}                      (st_ply_compressed_ply_file)
 *   compressedPlyTableToFile(cols, names,     processDataTable + writeCompressedPly of a host table
 *        actions, outFd, version)             into outFd (st_compressed_ply_file)
 *   sogBundleFromFile(fd, actions, iters,     readPly + processDataTable + writeSog -> .sog bytes,
 *        draws, dosTime, dosDate)             resident
 *        -> {archive, used}
 */
#define _GNU_SOURCE /* clock_gettime, madvise */
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/mman.h>
#include <time.h>

#include "st_abi.h"

static st_ctx *g_ctx = NULL;

#define NAPI_OK(call)                                                   \
    do {                                                                \
        if ((call) != napi_ok) {                                        \
            napi_throw_error(env, NULL, "splat-hip: N-API call failed"); \
            goto fail;                                                  \
        }                                                               \
    } while (0)

/* ST_DEBUG=1: where a long call's time goes, on stderr */
static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static napi_value throw_st(napi_env env, int rc) {
    char buf[600];
    char code[32];
    snprintf(buf, sizeof buf, "splat-hip: %s (status %d)", st_last_error(), rc);
    snprintf(code, sizeof code, "ST_STATUS_%d", -rc);  /* error.code: the st_status, tested by the host */
    napi_throw_error(env, code, buf);
    return NULL;
}

static int get_ctx(napi_env env, st_ctx **out) {
    if (!g_ctx) {
        int rc = st_ctx_create(0, &g_ctx);
        if (rc != ST_OK) {
            g_ctx = NULL;
            throw_st(env, rc);
            return 0;
        }
    }
    *out = g_ctx;
    return 1;
}

/* TypedArray storage of `v`; type-checked */
static void *ta_data(napi_env env, napi_value v, napi_typedarray_type want, size_t *len) {
    bool is_ta = false;
    napi_typedarray_type type;
    size_t length = 0, off = 0;
    void *data = NULL;
    napi_value ab;
    if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta ||
        napi_get_typedarray_info(env, v, &type, &length, &data, &ab, &off) != napi_ok || type != want) {
        napi_throw_type_error(env, NULL, "splat-hip: wrong TypedArray type");
        return NULL;
    }
    if (len) *len = length;
    return data;
}

static double num(napi_env env, napi_value v) {
    double d = 0;
    napi_get_value_double(env, v, &d);
    return d;
}

/* array of Float32Array -> float* list (caller frees); n = common length */
static float **f32_list(napi_env env, napi_value arr, uint32_t *count, uint64_t *n) {
    uint32_t m = 0;
    if (napi_get_array_length(env, arr, &m) != napi_ok) {
        napi_throw_type_error(env, NULL, "splat-hip: expected an array of Float32Array columns");
        return NULL;
    }
    float **p = (float **)calloc(m ? m : 1, sizeof(float *));
    *n = 0;
    for (uint32_t i = 0; i < m; ++i) {
        napi_value e;
        size_t len = 0;
        napi_get_element(env, arr, i, &e);
        p[i] = (float *)ta_data(env, e, napi_float32_array, &len);
        if (!p[i]) {
            free(p);
            return NULL;
        }
        if (i == 0) *n = len;
        else if (len != *n) {
            free(p);
            napi_throw_range_error(env, NULL, "splat-hip: columns differ in length");
            return NULL;
        }
    }
    *count = m;
    return p;
}

static void free_strs(char **s, uint32_t m);

/* a JS string as a NUL-terminated heap copy; NULL (TypeError thrown) when v is not a string */
static char *dup_str(napi_env env, napi_value v, const char *what) {
    size_t len = 0;
    char *s;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &len) != napi_ok) {
        napi_throw_type_error(env, NULL, what);
        return NULL;
    }
    s = (char *)malloc(len + 1);
    if (napi_get_value_string_utf8(env, v, s, len + 1, &len) != napi_ok) {
        free(s);
        napi_throw_type_error(env, NULL, what);
        return NULL;
    }
    s[len] = 0;
    return s;
}

/* array of m strings (caller frees); NULL (TypeError thrown) when an element is not a string */
static char **str_list(napi_env env, napi_value arr, uint32_t m) {
    char **s = (char **)calloc(m ? m : 1, sizeof(char *));
    for (uint32_t i = 0; i < m; ++i) {
        napi_value e;
        if (napi_get_element(env, arr, i, &e) != napi_ok ||
            !(s[i] = dup_str(env, e, "splat-hip: column names must be strings"))) {
            free_strs(s, i);
            return NULL;
        }
    }
    return s;
}

static void free_strs(char **s, uint32_t m) {
    if (!s) return;
    for (uint32_t i = 0; i < m; ++i) free(s[i]);
    free(s);
}

static napi_value new_typed(napi_env env, napi_typedarray_type type, size_t elems, size_t esize, void **data) {
    napi_value ab, ta;
    if (napi_create_arraybuffer(env, elems * esize, data, &ab) != napi_ok) return NULL;
    if (napi_create_typedarray(env, type, elems, ab, 0, &ta) != napi_ok) return NULL;
    return ta;
}

static void set_named(napi_env env, napi_value obj, const char *k, napi_value v) {
    napi_set_named_property(env, obj, k, v);
}

/* a large output column: its own 2 MiB-aligned allocation with transparent huge pages, handed to
 * JS as an external ArrayBuffer (freed by its finalizer).  V8's own ArrayBuffers are zero-filled
 * 4 KiB pages; the reader overwrites every byte anyway, and first-touch faults on 2.5 GB of 4 KiB
 * pages halved the rate of readPly's device-to-host copies. */
/* Freed columns' blocks are kept (up to ST_NAPI_POOL_MB, default 4096 MiB) and handed to the
 * next column of the same rounded length: a reused block is already faulted in, while a fresh
 * one is zeroed by the kernel on first touch inside the device-to-host copy (1,240 huge pages
 * for a 10M-splat table).  The pool is process-wide: with the addon loaded in worker_threads
 * each env's finalizers and allocations run on that env's own thread, so g_pool_mu guards it. */
#define POOL_MAX 512
static struct {
    void *p;
    size_t len;
} g_pool[POOL_MAX];
static int g_pool_n = 0;
static size_t g_pool_bytes = 0;
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;

static size_t pool_cap(void) {
    static size_t cap = (size_t)-1;
    if (cap == (size_t)-1) {
        const char *e = getenv("ST_NAPI_POOL_MB");
        cap = (size_t)(e ? strtoull(e, NULL, 10) : 4096) << 20;
    }
    return cap;
}

static void free_column(napi_env env, void *data, void *hint) {
    int64_t adj;
    const size_t bytes = (size_t)hint, huge = (size_t)2 << 20, len = (bytes + huge - 1) / huge * huge;
    napi_adjust_external_memory(env, -(int64_t)bytes, &adj);
    /* a resident readPly column (or a mirrored one) stops being one before its memory is reused */
    if (g_ctx) st_ply_forget(g_ctx, data);
    pthread_mutex_lock(&g_pool_mu);
    if (g_pool_n < POOL_MAX && g_pool_bytes + len <= pool_cap()) {
        g_pool[g_pool_n].p = data;
        g_pool[g_pool_n].len = len;
        ++g_pool_n;
        g_pool_bytes += len;
        pthread_mutex_unlock(&g_pool_mu);
        return;
    }
    pthread_mutex_unlock(&g_pool_mu);
    free(data);
}

/* always the external form (a resident readPly column needs the finalizer whatever its size) */
static napi_value new_typed_ext(napi_env env, napi_typedarray_type type, size_t elems, size_t esize, void **data) {
    const size_t bytes = elems * esize, huge = (size_t)2 << 20;
    if (!bytes) return new_typed(env, type, elems, esize, data);
    void *p = NULL;
    const size_t len = (bytes + huge - 1) / huge * huge;
    pthread_mutex_lock(&g_pool_mu);
    for (int i = g_pool_n - 1; i >= 0 && !p; --i)
        if (g_pool[i].len == len) {
            p = g_pool[i].p;
            g_pool[i] = g_pool[--g_pool_n];
            g_pool_bytes -= len;
        }
    pthread_mutex_unlock(&g_pool_mu);
    if (!p) {
        if (posix_memalign(&p, huge, len) != 0) {
            napi_throw_error(env, NULL, "splat-hip: out of host memory for a column");
            return NULL;
        }
        madvise(p, len, MADV_HUGEPAGE);  /* best effort */
    }
    napi_value ab, ta;
    if (napi_create_external_arraybuffer(env, p, bytes, free_column, (void *)bytes, &ab) != napi_ok) {
        free(p);
        return NULL;
    }
    int64_t adj;
    napi_adjust_external_memory(env, (int64_t)bytes, &adj);
    if (napi_create_typedarray(env, type, elems, ab, 0, &ta) != napi_ok) return NULL;
    *data = p;
    return ta;
}

static napi_value new_typed_big(napi_env env, napi_typedarray_type type, size_t elems, size_t esize, void **data) {
    if (elems * esize < ((size_t)8 << 20)) return new_typed(env, type, elems, esize, data);
    return new_typed_ext(env, type, elems, esize, data);
}

static napi_value make_num(napi_env env, double d) {
    napi_value v;
    napi_create_double(env, d, &v);
    return v;
}

/* ---- exports -------------------------------------------------------------- */
static napi_value js_version(napi_env env, napi_callback_info info) {
    (void)info;
    return make_num(env, st_abi_version());
}

/* rcclInfo() -> {version, path}: the RCCL the library's collectives run on (st_rccl_info) */
static napi_value js_rccl_info(napi_env env, napi_callback_info info) {
    (void)info;
    int32_t v = 0;
    char path[4096];
    napi_value out, s;
    const int rc = st_rccl_info(&v, path, sizeof path);
    if (rc != ST_OK) return throw_st(env, rc);
    NAPI_OK(napi_create_object(env, &out));
    set_named(env, out, "version", make_num(env, v));
    NAPI_OK(napi_create_string_utf8(env, path, NAPI_AUTO_LENGTH, &s));
    set_named(env, out, "path", s);
    return out;
fail:
    return NULL;
}

/* lastHostReuse() -> {columns, bytes}: how much of the last writeSog host form ran from readPly's
 * resident device columns (st_ctx_last_host_reuse; 0 = uploaded) */
static napi_value js_last_host_reuse(napi_env env, napi_callback_info info) {
    (void)info;
    st_ctx *ctx;
    uint64_t cols = 0, bytes = 0;
    napi_value out;
    if (!get_ctx(env, &ctx)) return NULL;
    const int rc = st_ctx_last_host_reuse(ctx, &cols, &bytes);
    if (rc != ST_OK) return throw_st(env, rc);
    NAPI_OK(napi_create_object(env, &out));
    set_named(env, out, "columns", make_num(env, (double)cols));
    set_named(env, out, "bytes", make_num(env, (double)bytes));
    return out;
fail:
    return NULL;
}

static napi_value js_device_count(napi_env env, napi_callback_info info) {
    (void)info;
    int32_t n = 0;
    if (st_device_count(&n) != ST_OK) n = 0;
    return make_num(env, n);
}

static napi_value js_quat_from_euler(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], out;
    double q[4];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    st_quat_from_euler(num(env, argv[0]), num(env, argv[1]), num(env, argv[2]), q);
    NAPI_OK(napi_create_array_with_length(env, 4, &out));
    for (uint32_t i = 0; i < 4; ++i) napi_set_element(env, out, i, make_num(env, q[i]));
    return out;
fail:
    return NULL;
}

/* transform(cols, names, t[3], r[4], s): mutates the Float32Array columns in place */
static napi_value js_transform(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5], e;
    uint32_t m = 0;
    uint64_t n = 0;
    float **cols = NULL;
    char **names = NULL;
    st_ctx *ctx;
    double t[3], r[4];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &m, &n))) return NULL;
    if (!(names = str_list(env, argv[1], m))) goto fail;
    for (uint32_t i = 0; i < 3; ++i) {
        napi_get_element(env, argv[2], i, &e);
        t[i] = num(env, e);
    }
    for (uint32_t i = 0; i < 4; ++i) {
        napi_get_element(env, argv[3], i, &e);
        r[i] = num(env, e);
    }
    {
        st_transform_params p;
        st_table tab = {n, (int32_t)m, (const char *const *)names, cols};
        int rc = st_transform_params_make(t, r, num(env, argv[4]), &p);
        if (rc == ST_OK && get_ctx(env, &ctx)) rc = st_transform(ctx, &tab, &p);
        else if (rc == ST_OK) goto fail;
        free(cols);
        free_strs(names, m);
        if (rc != ST_OK) return throw_st(env, rc);
    }
    return NULL;
fail:
    free(cols);
    free_strs(names, m);
    return NULL;
}

static napi_value js_filter_finite(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], out;
    uint32_t m = 0;
    uint64_t n = 0, kept = 0;
    float **cols;
    st_ctx *ctx;
    void *buf;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &m, &n))) return NULL;
    {
        uint32_t *idx = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
        st_table tab = {n, (int32_t)m, NULL, cols};
        int rc = get_ctx(env, &ctx) ? st_filter_finite(ctx, &tab, idx, &kept) : 1;
        free(cols);
        if (rc != ST_OK) {
            free(idx);
            return rc == 1 ? NULL : throw_st(env, rc);
        }
        out = new_typed(env, napi_uint32_array, kept, 4, &buf);
        memcpy(buf, idx, kept * 4);
        free(idx);
    }
    return out;
fail:
    return NULL;
}

/* setDevices(n): writeSog (sog / sogBundle) shards its rows over GPUs 0..n-1 (st_set_devices) */
static napi_value js_set_devices(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    {
        const int rc = st_set_devices((int32_t)num(env, argv[0]));
        if (rc != ST_OK) return throw_st(env, rc);
    }
    return NULL;
fail:
    return NULL;
}

static napi_value js_get_devices(napi_env env, napi_callback_info info) {
    int32_t n = 1;
    (void)info;
    st_get_devices(&n);
    return make_num(env, n);
}

/* TypedArray element type -> st_ply_type (0: not one of the reference's eight) */
static int ply_type_of(napi_typedarray_type t, size_t *esize) {
    switch (t) {
        case napi_int8_array: *esize = 1; return ST_PLY_CHAR;
        case napi_uint8_array: *esize = 1; return ST_PLY_UCHAR;
        case napi_int16_array: *esize = 2; return ST_PLY_SHORT;
        case napi_uint16_array: *esize = 2; return ST_PLY_USHORT;
        case napi_int32_array: *esize = 4; return ST_PLY_INT;
        case napi_uint32_array: *esize = 4; return ST_PLY_UINT;
        case napi_float32_array: *esize = 4; return ST_PLY_FLOAT;
        case napi_float64_array: *esize = 8; return ST_PLY_DOUBLE;
        default: *esize = 0; return 0;
    }
}

/* filterNaN(columns: TypedArray[]) -> TypedArray[] of the rows whose every value isFinite
 * (process.ts:84-95 -> filter -> permuteRows): one upload, compaction on the device, each
 * result column of its source's type (st_filter_nan) */
static napi_value js_filter_nan(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], out = NULL;
    uint32_t m = 0;
    uint64_t n = 0, kept = 0;
    st_ctx *ctx;
    void **src = NULL, **dst = NULL;
    int32_t *types = NULL;
    napi_typedarray_type *nt = NULL;
    size_t *es = NULL;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    NAPI_OK(napi_get_array_length(env, argv[0], &m));
    src = (void **)calloc(m + 1, sizeof(void *));
    dst = (void **)calloc(m + 1, sizeof(void *));
    types = (int32_t *)calloc(m + 1, sizeof(int32_t));
    nt = (napi_typedarray_type *)calloc(m + 1, sizeof(napi_typedarray_type));
    es = (size_t *)calloc(m + 1, sizeof(size_t));
    for (uint32_t i = 0; i < m; ++i) {
        napi_value e, ab;
        bool is_ta = false;
        size_t len = 0, off = 0;
        NAPI_OK(napi_get_element(env, argv[0], i, &e));
        if (napi_is_typedarray(env, e, &is_ta) != napi_ok || !is_ta ||
            napi_get_typedarray_info(env, e, &nt[i], &len, &src[i], &ab, &off) != napi_ok ||
            !(types[i] = ply_type_of(nt[i], &es[i]))) {
            napi_throw_type_error(env, NULL, "splat-hip: filterNaN expects the reference's TypedArray columns");
            goto fail;
        }
        if (i == 0) n = len;
        else if (len != n) {
            napi_throw_range_error(env, NULL, "splat-hip: columns differ in length");
            goto fail;
        }
    }
    for (uint32_t i = 0; i < m; ++i) dst[i] = malloc(n * es[i] + 8);
    {
        st_ttable ts = {n, (int32_t)m, NULL, types, src};
        st_ttable td = {n, (int32_t)m, NULL, types, dst};
        const char **noname = (const char **)calloc(m + 1, sizeof(char *));
        for (uint32_t i = 0; i < m; ++i) noname[i] = "";
        ts.names = td.names = noname;
        int rc = get_ctx(env, &ctx) ? st_filter_nan(ctx, &ts, &td, &kept) : 1;
        free(noname);
        if (rc != ST_OK) {
            if (rc != 1) throw_st(env, rc);
            goto fail;
        }
    }
    NAPI_OK(napi_create_array_with_length(env, m, &out));
    for (uint32_t i = 0; i < m; ++i) {
        void *buf;
        napi_value ta = new_typed(env, nt[i], kept, es[i], &buf);
        if (!ta) goto fail;
        memcpy(buf, dst[i], kept * es[i]);
        NAPI_OK(napi_set_element(env, out, i, ta));
    }
    for (uint32_t i = 0; i < m; ++i) free(dst[i]);
    free(src); free(dst); free(types); free(nt); free(es);
    return out;
fail:
    if (dst)
        for (uint32_t i = 0; i < m; ++i) free(dst[i]);
    free(src); free(dst); free(types); free(nt); free(es);
    return NULL;
}

/* ---- processDataTable chain (st_process / st_compressed_ply) ----------------------------
 * columns: TypedArray[] of the reference's eight types, names: string[], actions: the host's
 * normalised list [{k, t[3], r[4], s, column, compare, value, bands}] (js/index.js) */
typedef struct {
    uint32_t m;
    uint64_t n;
    void **cols;
    int32_t *types;
    napi_typedarray_type *nt;
    size_t *es;
    char **names;
    uint32_t na;
    st_action *acts;
    char **acols;
} chain_args;

static void chain_free(chain_args *a) {
    free(a->cols); free(a->types); free(a->nt); free(a->es);
    free_strs(a->names, a->m);
    free_strs(a->acols, a->na);
    free(a->acts);
}

static double prop_num(napi_env env, napi_value obj, const char *k) {
    napi_value v;
    if (napi_get_named_property(env, obj, k, &v) != napi_ok) return 0;
    return num(env, v);
}

static int parse_actions(napi_env env, napi_value actions, chain_args *a);

static int chain_parse(napi_env env, napi_value cols, napi_value names, napi_value actions, chain_args *a) {
    memset(a, 0, sizeof *a);
    if (napi_get_array_length(env, cols, &a->m) != napi_ok || napi_get_array_length(env, actions, &a->na) != napi_ok) {
        napi_throw_type_error(env, NULL, "splat-hip: expected column and action arrays");
        return 0;
    }
    a->cols = (void **)calloc(a->m + 1, sizeof(void *));
    a->types = (int32_t *)calloc(a->m + 1, sizeof(int32_t));
    a->nt = (napi_typedarray_type *)calloc(a->m + 1, sizeof(napi_typedarray_type));
    a->es = (size_t *)calloc(a->m + 1, sizeof(size_t));
    for (uint32_t i = 0; i < a->m; ++i) {
        napi_value e, ab;
        bool is_ta = false;
        size_t len = 0, off = 0;
        napi_get_element(env, cols, i, &e);
        if (napi_is_typedarray(env, e, &is_ta) != napi_ok || !is_ta ||
            napi_get_typedarray_info(env, e, &a->nt[i], &len, &a->cols[i], &ab, &off) != napi_ok ||
            !(a->types[i] = ply_type_of(a->nt[i], &a->es[i]))) {
            napi_throw_type_error(env, NULL, "splat-hip: expected the reference's TypedArray columns");
            return 0;
        }
        if (i == 0) a->n = len;
        else if (len != a->n) {
            napi_throw_range_error(env, NULL, "splat-hip: columns differ in length");
            return 0;
        }
    }
    if (!(a->names = str_list(env, names, a->m))) return 0;
    return parse_actions(env, actions, a);
}

/* the normalised action list into a->acts (a->na set by the caller) */
static int parse_actions(napi_env env, napi_value actions, chain_args *a) {
    a->acts = (st_action *)calloc(a->na + 1, sizeof(st_action));
    a->acols = (char **)calloc(a->na + 1, sizeof(char *));
    for (uint32_t i = 0; i < a->na; ++i) {
        napi_value o, v;
        st_action *x = &a->acts[i];
        napi_get_element(env, actions, i, &o);
        x->kind = (int32_t)prop_num(env, o, "k");
        x->compare = (int32_t)prop_num(env, o, "compare");
        x->value = prop_num(env, o, "value");
        x->bands = (int32_t)prop_num(env, o, "bands");
        if (x->kind == ST_ACTION_FILTER_VALUE && napi_get_named_property(env, o, "column", &v) == napi_ok) {
            if (!(a->acols[i] = dup_str(env, v, "splat-hip: filterByValue needs a column name string"))) return 0;
            x->column = a->acols[i];
        }
        if (x->kind == ST_ACTION_TRANSFORM) {
            double t[3], r[4];
            napi_value tv, rv, e;
            napi_get_named_property(env, o, "t", &tv);
            napi_get_named_property(env, o, "r", &rv);
            for (uint32_t j = 0; j < 3; ++j) napi_get_element(env, tv, j, &e), t[j] = num(env, e);
            for (uint32_t j = 0; j < 4; ++j) napi_get_element(env, rv, j, &e), r[j] = num(env, e);
            int rc = st_transform_params_make(t, r, prop_num(env, o, "s"), &x->transform);
            if (rc != ST_OK) {
                throw_st(env, rc);
                return 0;
            }
        }
    }
    return 1;
}

/* compressedPly(columns, names, actions) -> {numRows, shCoeffs, chunk, vertex, sh}:
 * processDataTable then writeCompressedPly's arrays in one upload (st_compressed_ply) */
static napi_value js_compressed_ply(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], out = NULL;
    chain_args a;
    st_ctx *ctx;
    float *chunk = NULL;
    uint32_t *vertex = NULL;
    uint8_t *sh = NULL;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (!chain_parse(env, argv[0], argv[1], argv[2], &a)) goto fail;
    if (!get_ctx(env, &ctx)) goto fail;
    chunk = (float *)malloc(((a.n + 255) / 256 * 18 + 1) * 4);
    vertex = (uint32_t *)malloc((a.n * 4 + 1) * 4);
    sh = (uint8_t *)malloc(a.n * 45 + 1);
    {
        st_ttable ts = {a.n, (int32_t)a.m, (const char *const *)a.names, a.types, a.cols};
        uint64_t m = 0;
        int32_t C = 0;
        void *p;
        napi_value tch, tvx, tsh;
        int rc = st_compressed_ply(ctx, &ts, a.acts, (int32_t)a.na, chunk, vertex, sh, &m, &C);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        const uint64_t nch = (m + 255) / 256;
        if (!(tch = new_typed(env, napi_float32_array, nch * 18, 4, &p))) goto fail;
        memcpy(p, chunk, nch * 18 * 4);
        if (!(tvx = new_typed(env, napi_uint32_array, m * 4, 4, &p))) goto fail;
        memcpy(p, vertex, m * 16);
        if (!(tsh = new_typed(env, napi_uint8_array, m * 3 * (uint64_t)C, 1, &p))) goto fail;
        memcpy(p, sh, m * 3 * (uint64_t)C);
        if (napi_create_object(env, &out) != napi_ok) goto fail;
        set_named(env, out, "numRows", make_num(env, (double)m));
        set_named(env, out, "shCoeffs", make_num(env, C));
        set_named(env, out, "chunk", tch);
        set_named(env, out, "vertex", tvx);
        set_named(env, out, "sh", tsh);
    }
    free(chunk); free(vertex); free(sh);
    chain_free(&a);
    return out;
fail:
    free(chunk); free(vertex); free(sh);
    chain_free(&a);
    return NULL;
}

/* compressedPlyFromFile(fd, actions) -> {numRows, shCoeffs, chunk, vertex, sh}: readPly +
 * processDataTable + writeCompressedPly's arrays, the rows resident in HBM (st_ply_compressed_ply) */
static napi_value js_compressed_ply_file(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out = NULL;
    chain_args a;
    st_ctx *ctx;
    st_ply_header *h = NULL;
    float *chunk = NULL;
    uint32_t *vertex = NULL;
    uint8_t *sh = NULL;
    memset(&a, 0, sizeof a);
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (napi_get_array_length(env, argv[1], &a.na) != napi_ok || !parse_actions(env, argv[1], &a)) goto fail;
    if (!get_ctx(env, &ctx)) goto fail;
    h = (st_ply_header *)calloc(1, sizeof *h);
    {
        const int32_t fd = (int32_t)num(env, argv[0]);
        int rc = st_ply_read_header(fd, h), el = -1;
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        for (int e = 0; e < h->nelements && el < 0; ++e)
            if (strcmp(h->elements[e].name, "vertex") == 0) el = e;
        if (el < 0) {
            napi_throw_error(env, NULL, "splat-hip: no vertex element");
            goto fail;
        }
        const uint64_t n = h->elements[el].count;
        chunk = (float *)malloc(((n + 255) / 256 * 18 + 1) * 4);
        vertex = (uint32_t *)malloc((n * 4 + 1) * 4);
        sh = (uint8_t *)malloc(n * 45 + 1);
        uint64_t m = 0;
        int32_t C = 0;
        void *p;
        napi_value tch, tvx, tsh;
        rc = st_ply_compressed_ply(ctx, fd, h, el, a.acts, (int32_t)a.na, chunk, vertex, sh, &m, &C);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        const uint64_t nch = (m + 255) / 256;
        if (!(tch = new_typed(env, napi_float32_array, nch * 18, 4, &p))) goto fail;
        memcpy(p, chunk, nch * 18 * 4);
        if (!(tvx = new_typed(env, napi_uint32_array, m * 4, 4, &p))) goto fail;
        memcpy(p, vertex, m * 16);
        if (!(tsh = new_typed(env, napi_uint8_array, m * 3 * (uint64_t)C, 1, &p))) goto fail;
        memcpy(p, sh, m * 3 * (uint64_t)C);
        if (napi_create_object(env, &out) != napi_ok) goto fail;
        set_named(env, out, "numRows", make_num(env, (double)m));
        set_named(env, out, "shCoeffs", make_num(env, C));
        set_named(env, out, "chunk", tch);
        set_named(env, out, "vertex", tvx);
        set_named(env, out, "sh", tsh);
    }
    free(chunk); free(vertex); free(sh); free(h);
    chain_free(&a);
    return out;
fail:
    free(chunk); free(vertex); free(sh); free(h);
    chain_free(&a);
    return NULL;
}

/* compressedPlyToFile(inFd, actions, outFd, version) -> {numRows, shCoeffs, size}: readPly +
 * processDataTable + writeCompressedPly into outFd (st_ply_compressed_ply_file: the arrays written
 * at offsets as they leave HBM) */
static napi_value js_compressed_ply_to_file(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4], out = NULL;
    chain_args a;
    st_ctx *ctx;
    st_ply_header *h = NULL;
    char *version = NULL;
    memset(&a, 0, sizeof a);
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (napi_get_array_length(env, argv[1], &a.na) != napi_ok || !parse_actions(env, argv[1], &a)) goto fail;
    if (argc > 3 && !(version = dup_str(env, argv[3], "splat-hip: version must be a string"))) goto fail;
    if (!get_ctx(env, &ctx)) goto fail;
    h = (st_ply_header *)calloc(1, sizeof *h);
    {
        const int32_t fd = (int32_t)num(env, argv[0]), ofd = (int32_t)num(env, argv[2]);
        int rc = st_ply_read_header(fd, h), el = -1;
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        for (int e = 0; e < h->nelements && el < 0; ++e)
            if (strcmp(h->elements[e].name, "vertex") == 0) el = e;
        if (el < 0) {
            napi_throw_error(env, NULL, "splat-hip: no vertex element");
            goto fail;
        }
        uint64_t m = 0, size = 0;
        int32_t C = 0;
        rc = st_ply_compressed_ply_file(ctx, fd, h, el, a.acts, (int32_t)a.na, ofd, version, &m, &C, &size);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        if (napi_create_object(env, &out) != napi_ok) goto fail;
        set_named(env, out, "numRows", make_num(env, (double)m));
        set_named(env, out, "shCoeffs", make_num(env, C));
        set_named(env, out, "size", make_num(env, (double)size));
    }
    free(h);
    free(version);
    chain_free(&a);
    return out;
fail:
    free(h);
    free(version);
    chain_free(&a);
    return NULL;
}

/* compressedPlyTableToFile(columns, names, actions, outFd, version) -> {numRows, shCoeffs, size}:
 * processDataTable + writeCompressedPly of a host table into outFd (st_compressed_ply_file) */
static napi_value js_compressed_ply_table_to_file(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5], out = NULL;
    chain_args a;
    st_ctx *ctx;
    char *version = NULL;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (!chain_parse(env, argv[0], argv[1], argv[2], &a)) goto fail;
    if (argc > 4 && !(version = dup_str(env, argv[4], "splat-hip: version must be a string"))) goto fail;
    if (!get_ctx(env, &ctx)) goto fail;
    {
        st_ttable ts = {a.n, (int32_t)a.m, (const char *const *)a.names, a.types, a.cols};
        uint64_t m = 0, size = 0;
        int32_t C = 0;
        const int rc = st_compressed_ply_file(ctx, &ts, a.acts, (int32_t)a.na, (int32_t)num(env, argv[3]), version,
                                              &m, &C, &size);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        if (napi_create_object(env, &out) != napi_ok) goto fail;
        set_named(env, out, "numRows", make_num(env, (double)m));
        set_named(env, out, "shCoeffs", make_num(env, C));
        set_named(env, out, "size", make_num(env, (double)size));
    }
    free(version);
    chain_free(&a);
    return out;
fail:
    free(version);
    chain_free(&a);
    return NULL;
}

/* sogBundleFromFile(fd, actions, iters, draws: Float64Array, dosTime, dosDate) -> {archive, used}:
 * readPly + processDataTable + writeSog to .sog bytes, resident (st_ply_sog_bundle) */
static napi_value js_sog_bundle_file(napi_env env, napi_callback_info info) {
    size_t argc = 6, nd = 0;
    napi_value argv[6], out = NULL, buf;
    chain_args a;
    st_ctx *ctx;
    st_ply_header *h = NULL;
    uint8_t *arch = NULL;
    uint64_t size = 0, used = 0;
    memset(&a, 0, sizeof a);
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (napi_get_array_length(env, argv[1], &a.na) != napi_ok || !parse_actions(env, argv[1], &a)) goto fail;
    {
        double *draws = (double *)ta_data(env, argv[3], napi_float64_array, &nd);
        if (!draws || !get_ctx(env, &ctx)) goto fail;
        h = (st_ply_header *)calloc(1, sizeof *h);
        const int32_t fd = (int32_t)num(env, argv[0]);
        int rc = st_ply_read_header(fd, h);
        if (rc == ST_OK)
            rc = st_ply_sog_bundle(ctx, fd, h, -1, a.acts, (int32_t)a.na, (int32_t)num(env, argv[2]), draws, nd, &used,
                                   (uint16_t)num(env, argv[4]), (uint16_t)num(env, argv[5]), &arch, &size);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        void *p;
        if (napi_create_buffer_copy(env, size, arch, &p, &buf) != napi_ok) goto fail;
        if (napi_create_object(env, &out) != napi_ok) goto fail;
        set_named(env, out, "archive", buf);
        set_named(env, out, "used", make_num(env, (double)used));
    }
    st_free(arch);
    free(h);
    chain_free(&a);
    return out;
fail:
    st_free(arch);
    free(h);
    chain_free(&a);
    return NULL;
}

/* process(columns, names, actions, outNames, outSrc) -> TypedArray[]: processDataTable in one
 * upload (st_process); result column j is named outNames[j] and has the type of source column
 * outSrc[j] (the host computes filterBands' renaming) */
static napi_value js_process(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5], out = NULL;
    chain_args a;
    st_ctx *ctx;
    uint32_t mo = 0;
    char **onames = NULL;
    void **dst = NULL;
    int32_t *otypes = NULL;
    uint32_t *osrc = NULL;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (!chain_parse(env, argv[0], argv[1], argv[2], &a)) goto fail;
    if (napi_get_array_length(env, argv[3], &mo) != napi_ok) goto fail;
    if (!(onames = str_list(env, argv[3], mo))) goto fail;
    dst = (void **)calloc(mo + 1, sizeof(void *));
    otypes = (int32_t *)calloc(mo + 1, sizeof(int32_t));
    osrc = (uint32_t *)calloc(mo + 1, sizeof(uint32_t));
    for (uint32_t j = 0; j < mo; ++j) {
        napi_value e;
        napi_get_element(env, argv[4], j, &e);
        osrc[j] = (uint32_t)num(env, e);
        if (osrc[j] >= a.m) {
            napi_throw_range_error(env, NULL, "splat-hip: bad result column source");
            goto fail;
        }
        otypes[j] = a.types[osrc[j]];
        dst[j] = malloc(a.n * a.es[osrc[j]] + 8);
    }
    if (!get_ctx(env, &ctx)) goto fail;
    {
        st_ttable ts = {a.n, (int32_t)a.m, (const char *const *)a.names, a.types, a.cols};
        st_ttable td = {a.n, (int32_t)mo, (const char *const *)onames, otypes, dst};
        uint64_t m = 0;
        int rc = st_process(ctx, &ts, a.acts, (int32_t)a.na, &td, &m);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        if (napi_create_array_with_length(env, mo, &out) != napi_ok) goto fail;
        for (uint32_t j = 0; j < mo; ++j) {
            void *buf;
            const size_t es = a.es[osrc[j]];
            napi_value ta = new_typed(env, a.nt[osrc[j]], m, es, &buf);
            if (!ta) goto fail;
            memcpy(buf, dst[j], m * es);
            napi_set_element(env, out, j, ta);
        }
    }
    for (uint32_t j = 0; j < mo; ++j) free(dst[j]);
    free(dst); free(otypes); free(osrc);
    free_strs(onames, mo);
    chain_free(&a);
    return out;
fail:
    if (dst)
        for (uint32_t j = 0; j < mo; ++j) free(dst[j]);
    free(dst); free(otypes); free(osrc);
    free_strs(onames, mo);
    chain_free(&a);
    return NULL;
}

/* combineLayout(tables: [{names: string[], types: number[]}]) -> [[table, column], ...]:
 * combine()'s result columns (index.ts:164-178, st_combine_layout) */
static napi_value js_combine_layout(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], out = NULL;
    uint32_t nt = 0;
    st_ttable *tabs = NULL;
    const st_ttable **ptrs = NULL;
    char ***names = NULL;
    int32_t **types = NULL;
    uint32_t *ncols = NULL;
    int32_t *ct = NULL, *ci = NULL, nout = 0;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    NAPI_OK(napi_get_array_length(env, argv[0], &nt));
    tabs = (st_ttable *)calloc(nt + 1, sizeof(st_ttable));
    ptrs = (const st_ttable **)calloc(nt + 1, sizeof(st_ttable *));
    names = (char ***)calloc(nt + 1, sizeof(char **));
    types = (int32_t **)calloc(nt + 1, sizeof(int32_t *));
    ncols = (uint32_t *)calloc(nt + 1, sizeof(uint32_t));
    for (uint32_t t = 0; t < nt; ++t) {
        napi_value tab, nv, tv, e;
        NAPI_OK(napi_get_element(env, argv[0], t, &tab));
        NAPI_OK(napi_get_named_property(env, tab, "names", &nv));
        NAPI_OK(napi_get_named_property(env, tab, "types", &tv));
        NAPI_OK(napi_get_array_length(env, nv, &ncols[t]));
        if (!(names[t] = str_list(env, nv, ncols[t]))) goto fail;
        types[t] = (int32_t *)calloc(ncols[t] + 1, sizeof(int32_t));
        for (uint32_t j = 0; j < ncols[t]; ++j) {
            NAPI_OK(napi_get_element(env, tv, j, &e));
            types[t][j] = (int32_t)num(env, e);
        }
        tabs[t].ncol = (int32_t)ncols[t];
        tabs[t].names = (const char *const *)names[t];
        tabs[t].types = types[t];
        ptrs[t] = &tabs[t];
    }
    {
        int rc = st_combine_layout(ptrs, (int32_t)nt, NULL, NULL, &nout);
        if (rc == ST_OK) {
            ct = (int32_t *)calloc(nout + 1, sizeof(int32_t));
            ci = (int32_t *)calloc(nout + 1, sizeof(int32_t));
            rc = st_combine_layout(ptrs, (int32_t)nt, ct, ci, &nout);
        }
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
    }
    NAPI_OK(napi_create_array_with_length(env, nout, &out));
    for (int32_t i = 0; i < nout; ++i) {
        napi_value pair;
        NAPI_OK(napi_create_array_with_length(env, 2, &pair));
        NAPI_OK(napi_set_element(env, pair, 0, make_num(env, ct[i])));
        NAPI_OK(napi_set_element(env, pair, 1, make_num(env, ci[i])));
        NAPI_OK(napi_set_element(env, out, i, pair));
    }
fail:
    for (uint32_t t = 0; t < nt; ++t) {
        free_strs(names ? names[t] : NULL, ncols ? ncols[t] : 0);
        if (types) free(types[t]);
    }
    free(tabs); free(ptrs); free(names); free(types); free(ncols); free(ct); free(ci);
    return out;
}

/* mortonOrder(x, y, z, indices): reorders `indices` in place, returns it */
static napi_value js_morton(napi_env env, napi_callback_info info) {
    size_t argc = 4, nx = 0, ny = 0, nz = 0, ni = 0;
    napi_value argv[4];
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    {
        float *x = (float *)ta_data(env, argv[0], napi_float32_array, &nx);
        float *y = (float *)ta_data(env, argv[1], napi_float32_array, &ny);
        float *z = (float *)ta_data(env, argv[2], napi_float32_array, &nz);
        uint32_t *idx = (uint32_t *)ta_data(env, argv[3], napi_uint32_array, &ni);
        if (!x || !y || !z || !idx) return NULL;
        if (nx != ny || nx != nz || ni != nx) {
            /* writeCompressedPly / writeSog order all rows (write-compressed-ply.ts:61-65, write-sog.ts:42-49) */
            napi_throw_range_error(env, NULL, "splat-hip: x/y/z/indices lengths differ");
            return NULL;
        }
        if (!get_ctx(env, &ctx)) return NULL;
        int rc = st_morton_order(ctx, x, y, z, idx, (uint64_t)ni);
        if (rc != ST_OK) return throw_st(env, rc);
    }
    return argv[3];
fail:
    return NULL;
}

static napi_value js_pack_compressed(napi_env env, napi_callback_info info) {
    size_t argc = 4, no = 0;
    napi_value argv[4], out;
    uint32_t m = 0;
    uint64_t n = 0;
    float **cols = NULL;
    char **names = NULL;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &m, &n))) return NULL;
    if (!(names = str_list(env, argv[1], m))) goto fail;
    {
        uint32_t *order = (uint32_t *)ta_data(env, argv[2], napi_uint32_array, &no);
        int32_t nsh = (int32_t)num(env, argv[3]);
        void *chunk, *vertex, *sh;
        const uint64_t nch = (no + 255) / 256;
        napi_value tch, tvx, tsh;
        if (!order) goto fail;
        if (no != n) {
            napi_throw_range_error(env, NULL, "splat-hip: order must name every row");
            goto fail;
        }
        tch = new_typed(env, napi_float32_array, nch * 18, 4, &chunk);
        tvx = new_typed(env, napi_uint32_array, no * 4, 4, &vertex);
        tsh = new_typed(env, napi_uint8_array, no * (uint64_t)nsh, 1, &sh);
        if (!get_ctx(env, &ctx)) goto fail;
        {
            st_table tab = {n, (int32_t)m, (const char *const *)names, cols};
            int rc = st_pack_compressed(ctx, &tab, order, (float *)chunk, (uint32_t *)vertex, (uint8_t *)sh);
            if (rc != ST_OK) {
                free(cols);
                free_strs(names, m);
                return throw_st(env, rc);
            }
        }
        NAPI_OK(napi_create_object(env, &out));
        set_named(env, out, "chunk", tch);
        set_named(env, out, "vertex", tvx);
        set_named(env, out, "sh", tsh);
    }
    free(cols);
    free_strs(names, m);
    return out;
fail:
    free(cols);
    free_strs(names, m);
    return NULL;
}

static napi_value js_kmeans(napi_env env, napi_callback_info info) {
    size_t argc = 4, nd = 0;
    napi_value argv[4], out;
    uint32_t d = 0;
    uint64_t n = 0, used = 0;
    float **cols;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &d, &n))) return NULL;
    {
        const int32_t k = (int32_t)num(env, argv[1]), iters = (int32_t)num(env, argv[2]);
        double *draws = (double *)ta_data(env, argv[3], napi_float64_array, &nd);
        const uint64_t kk = (uint64_t)k < n ? (uint64_t)k : n;
        void *cen, *lab;
        napi_value tc, tl;
        if (!draws) {
            free(cols);
            return NULL;
        }
        tc = new_typed(env, napi_float32_array, kk * d, 4, &cen);
        tl = new_typed(env, napi_uint32_array, n, 4, &lab);
        if (!get_ctx(env, &ctx)) {
            free(cols);
            return NULL;
        }
        int rc = st_kmeans(ctx, (const float *const *)cols, (int32_t)d, n, k, iters, draws, nd, &used, (float *)cen,
                           (uint32_t *)lab);
        free(cols);
        if (rc != ST_OK) return throw_st(env, rc);
        NAPI_OK(napi_create_object(env, &out));
        set_named(env, out, "centroids", tc); /* column-major: d columns of kk values */
        set_named(env, out, "labels", tl);
        set_named(env, out, "used", make_num(env, (double)used));
    }
    return out;
fail:
    return NULL;
}

static napi_value js_cluster1d(napi_env env, napi_callback_info info) {
    size_t argc = 3, nd = 0;
    napi_value argv[3], out;
    uint32_t m = 0;
    uint64_t n = 0, used = 0;
    float **cols;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &m, &n))) return NULL;
    {
        const int32_t iters = (int32_t)num(env, argv[1]);
        double *draws = (double *)ta_data(env, argv[2], napi_float64_array, &nd);
        void *cen, *lab;
        napi_value tc, tl;
        if (!draws) {
            free(cols);
            return NULL;
        }
        tc = new_typed(env, napi_float32_array, 256, 4, &cen);
        tl = new_typed(env, napi_uint8_array, n * m, 1, &lab);
        if (!get_ctx(env, &ctx)) {
            free(cols);
            return NULL;
        }
        int rc = st_cluster1d(ctx, (const float *const *)cols, (int32_t)m, n, iters, draws, nd, &used, (float *)cen,
                              (uint8_t *)lab);
        free(cols);
        if (rc != ST_OK) return throw_st(env, rc);
        NAPI_OK(napi_create_object(env, &out));
        set_named(env, out, "centroids", tc);
        set_named(env, out, "labels", tl); /* m column blocks of n bytes */
        set_named(env, out, "used", make_num(env, (double)used));
    }
    return out;
fail:
    return NULL;
}

static napi_value f32_copy(napi_env env, const float *src, size_t n) {
    void *d;
    napi_value v = new_typed(env, napi_float32_array, n, 4, &d);
    memcpy(d, src, n * 4);
    return v;
}

static napi_value js_sog(napi_env env, napi_callback_info info) {
    size_t argc = 4, nd = 0;
    napi_value argv[4], out, tex;
    uint32_t m = 0;
    uint64_t n = 0, used = 0;
    float **cols = NULL;
    char **names = NULL;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &m, &n))) return NULL;
    if (!(names = str_list(env, argv[1], m))) goto fail;
    {
        const int32_t iters = (int32_t)num(env, argv[2]);
        double *draws = (double *)ta_data(env, argv[3], napi_float64_array, &nd);
        int32_t W = 0, H = 0, pal = 0, cw = 0, ch = 0, sh = 0;
        st_sog_meta meta;
        st_sog_textures t;
        void *p[7];
        napi_value tv[7];
        static const char *tn[7] = {"means_l", "means_u", "quats", "scales", "sh0", "shN_centroids", "shN_labels"};
        if (!draws) goto fail;
        for (uint32_t i = 0; i < m; ++i)
            if (strcmp(names[i], "f_rest_44") == 0) sh = 15;
            else if (strcmp(names[i], "f_rest_23") == 0 && sh < 8) sh = 8;
            else if (strcmp(names[i], "f_rest_8") == 0 && sh < 3) sh = 3;
        if (st_sog_geometry(n, sh, &W, &H, &pal, &cw, &ch) != ST_OK) {
            napi_throw_range_error(env, NULL, "splat-hip: empty table");
            goto fail;
        }
        for (int i = 0; i < 7; ++i) {
            const size_t bytes = (i == 5) ? (size_t)cw * ch * 4 : (size_t)W * H * 4;
            tv[i] = new_typed(env, napi_uint8_array, bytes, 1, &p[i]);
        }
        t.means_l = (uint8_t *)p[0];
        t.means_u = (uint8_t *)p[1];
        t.quats = (uint8_t *)p[2];
        t.scales = (uint8_t *)p[3];
        t.sh0 = (uint8_t *)p[4];
        t.shn_centroids = cw ? (uint8_t *)p[5] : NULL;
        t.shn_labels = cw ? (uint8_t *)p[6] : NULL;
        if (!get_ctx(env, &ctx)) goto fail;
        {
            st_table tab = {n, (int32_t)m, (const char *const *)names, cols};
            int rc = st_sog(ctx, &tab, iters, draws, nd, &used, &meta, &t);
            if (rc != ST_OK) {
                free(cols);
                free_strs(names, m);
                return throw_st(env, rc);
            }
        }
        NAPI_OK(napi_create_object(env, &out));
        NAPI_OK(napi_create_object(env, &tex));
        for (int i = 0; i < 7; ++i)
            if (i < 5 || cw) set_named(env, tex, tn[i], tv[i]);
        set_named(env, out, "textures", tex);
        set_named(env, out, "width", make_num(env, meta.width));
        set_named(env, out, "height", make_num(env, meta.height));
        {
            napi_value mins, maxs;
            napi_create_array_with_length(env, 3, &mins);
            napi_create_array_with_length(env, 3, &maxs);
            for (uint32_t i = 0; i < 3; ++i) {
                napi_set_element(env, mins, i, make_num(env, meta.means_min[i]));
                napi_set_element(env, maxs, i, make_num(env, meta.means_max[i]));
            }
            set_named(env, out, "meansMins", mins);
            set_named(env, out, "meansMaxs", maxs);
        }
        set_named(env, out, "scalesCodebook", f32_copy(env, meta.scales_codebook, 256));
        set_named(env, out, "sh0Codebook", f32_copy(env, meta.sh0_codebook, 256));
        set_named(env, out, "shBands", make_num(env, meta.sh_bands));
        set_named(env, out, "paletteSize", make_num(env, meta.palette_size));
        set_named(env, out, "shNCodebook", f32_copy(env, meta.shn_codebook, 256));
        set_named(env, out, "shNWidth", make_num(env, meta.shn_width));
        set_named(env, out, "shNHeight", make_num(env, meta.shn_height));
        set_named(env, out, "used", make_num(env, (double)used));
    }
    free(cols);
    free_strs(names, m);
    return out;
fail:
    free(cols);
    free_strs(names, m);
    return NULL;
}

/* the band rule of the reference (write-sog.ts:296) over column names */
static int32_t sh_coeffs_of_names(char **names, uint32_t m) {
    int first_missing = -1;
    char nm[16];
    for (int i = 0; i < 45 && first_missing < 0; ++i) {
        int hit = 0;
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        for (uint32_t j = 0; j < m && !hit; ++j) hit = strcmp(names[j], nm) == 0;
        if (!hit) first_missing = i;
    }
    return first_missing == 9 ? 3 : first_missing == 24 ? 8 : first_missing == -1 ? 15 : 0;
}

/* sogProcess(columns: TypedArray[] of any of the eight types, names, actions, iters, draws) ->
 * as sog(): processDataTable then writeSog's textures and meta (st_sog_process) */
static napi_value js_sog_process(napi_env env, napi_callback_info info) {
    size_t argc = 5, nd = 0;
    napi_value argv[5], out = NULL, tex;
    chain_args a;
    st_ctx *ctx;
    uint8_t *hb[7] = {NULL, NULL, NULL, NULL, NULL, NULL, NULL};
    static const char *tn[7] = {"means_l", "means_u", "quats", "scales", "sh0", "shN_centroids", "shN_labels"};
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (!chain_parse(env, argv[0], argv[1], argv[2], &a)) goto fail;
    {
        const int32_t iters = (int32_t)num(env, argv[3]);
        double *draws = (double *)ta_data(env, argv[4], napi_float64_array, &nd);
        int32_t W = 0, H = 0, pal = 0, cw = 0, ch = 0;
        uint64_t used = 0;
        st_sog_meta meta;
        st_sog_textures t;
        if (!draws || !get_ctx(env, &ctx)) goto fail;
        /* sized for the input rows and band (the actions only remove rows or bands) */
        if (st_sog_geometry(a.n, sh_coeffs_of_names(a.names, a.m), &W, &H, &pal, &cw, &ch) != ST_OK) {
            napi_throw_range_error(env, NULL, "splat-hip: empty table");
            goto fail;
        }
        for (int i = 0; i < 7; ++i) hb[i] = (uint8_t *)malloc(((i == 5) ? (size_t)cw * ch * 4 : (size_t)W * H * 4) + 1);
        t.means_l = hb[0], t.means_u = hb[1], t.quats = hb[2], t.scales = hb[3], t.sh0 = hb[4];
        t.shn_centroids = hb[5], t.shn_labels = hb[6];
        {
            st_ttable ts = {a.n, (int32_t)a.m, (const char *const *)a.names, a.types, a.cols};
            int rc = st_sog_process(ctx, &ts, a.acts, (int32_t)a.na, iters, draws, nd, &used, &meta, &t);
            if (rc != ST_OK) {
                throw_st(env, rc);
                goto fail;
            }
        }
        {
            /* the processed table's geometry (its rows and band after the actions) */
            const int has_sh = meta.sh_bands > 0;
            if (napi_create_object(env, &out) != napi_ok || napi_create_object(env, &tex) != napi_ok) goto fail;
            for (int i = 0; i < 7; ++i) {
                const size_t b = (i == 5) ? (size_t)meta.shn_width * meta.shn_height * 4
                                          : (size_t)meta.width * meta.height * 4;
                void *p;
                napi_value v;
                if (i >= 5 && !has_sh) continue;
                if (!(v = new_typed(env, napi_uint8_array, b, 1, &p))) goto fail;
                memcpy(p, hb[i], b);
                set_named(env, tex, tn[i], v);
            }
        }
        set_named(env, out, "textures", tex);
        set_named(env, out, "width", make_num(env, meta.width));
        set_named(env, out, "height", make_num(env, meta.height));
        {
            napi_value mins, maxs;
            napi_create_array_with_length(env, 3, &mins);
            napi_create_array_with_length(env, 3, &maxs);
            for (uint32_t i = 0; i < 3; ++i) {
                napi_set_element(env, mins, i, make_num(env, meta.means_min[i]));
                napi_set_element(env, maxs, i, make_num(env, meta.means_max[i]));
            }
            set_named(env, out, "meansMins", mins);
            set_named(env, out, "meansMaxs", maxs);
        }
        set_named(env, out, "scalesCodebook", f32_copy(env, meta.scales_codebook, 256));
        set_named(env, out, "sh0Codebook", f32_copy(env, meta.sh0_codebook, 256));
        set_named(env, out, "shBands", make_num(env, meta.sh_bands));
        set_named(env, out, "paletteSize", make_num(env, meta.palette_size));
        set_named(env, out, "shNCodebook", f32_copy(env, meta.shn_codebook, 256));
        set_named(env, out, "shNWidth", make_num(env, meta.shn_width));
        set_named(env, out, "shNHeight", make_num(env, meta.shn_height));
        set_named(env, out, "used", make_num(env, (double)used));
    }
    for (int i = 0; i < 7; ++i) free(hb[i]);
    chain_free(&a);
    return out;
fail:
    for (int i = 0; i < 7; ++i) free(hb[i]);
    chain_free(&a);
    return NULL;
}

/* sogBundleProcess(columns: TypedArray[] of any type, names, actions, iters, draws, dosTime,
 * dosDate) -> {archive, used}: processDataTable then writeSog to .sog bytes (st_sog_bundle_process) */
static napi_value js_sog_bundle_process(napi_env env, napi_callback_info info) {
    size_t argc = 7, nd = 0;
    napi_value argv[7], out = NULL, buf;
    chain_args a;
    st_ctx *ctx;
    uint8_t *arch = NULL;
    uint64_t size = 0, used = 0;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (!chain_parse(env, argv[0], argv[1], argv[2], &a)) goto fail;
    {
        double *draws = (double *)ta_data(env, argv[4], napi_float64_array, &nd);
        if (!draws || !get_ctx(env, &ctx)) goto fail;
        st_ttable ts = {a.n, (int32_t)a.m, (const char *const *)a.names, a.types, a.cols};
        int rc = st_sog_bundle_process(ctx, &ts, a.acts, (int32_t)a.na, (int32_t)num(env, argv[3]), draws, nd, &used,
                                       (uint16_t)num(env, argv[5]), (uint16_t)num(env, argv[6]), &arch, &size);
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
        void *p;
        if (napi_create_buffer_copy(env, size, arch, &p, &buf) != napi_ok) goto fail;
        if (napi_create_object(env, &out) != napi_ok) goto fail;
        set_named(env, out, "archive", buf);
        set_named(env, out, "used", make_num(env, (double)used));
    }
    st_free(arch);
    chain_free(&a);
    return out;
fail:
    st_free(arch);
    chain_free(&a);
    return NULL;
}

/* transformTyped(columns: TypedArray[] of any type, names, t[3], r[4], s): transform() in place
 * (st_transform_t) */
static napi_value js_transform_typed(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5], e, none;
    chain_args a;
    st_ctx *ctx;
    double t[3], r[4];
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (napi_create_array_with_length(env, 0, &none) != napi_ok) return NULL;
    if (!chain_parse(env, argv[0], argv[1], none, &a)) goto fail;
    for (uint32_t i = 0; i < 3; ++i) napi_get_element(env, argv[2], i, &e), t[i] = num(env, e);
    for (uint32_t i = 0; i < 4; ++i) napi_get_element(env, argv[3], i, &e), r[i] = num(env, e);
    {
        st_transform_params p;
        st_ttable ts = {a.n, (int32_t)a.m, (const char *const *)a.names, a.types, a.cols};
        int rc = st_transform_params_make(t, r, num(env, argv[4]), &p);
        if (rc == ST_OK) {
            if (!get_ctx(env, &ctx)) goto fail;
            rc = st_transform_t(ctx, &ts, &p);
        }
        if (rc != ST_OK) {
            throw_st(env, rc);
            goto fail;
        }
    }
    chain_free(&a);
    return NULL;
fail:
    chain_free(&a);
    return NULL;
}

/* mortonOrderTyped(x, y, z: TypedArrays of any type, indices: Uint32Array) -> indices
 * (st_morton_order_t) */
static napi_value js_morton_typed(napi_env env, napi_callback_info info) {
    size_t argc = 4, ni = 0;
    napi_value argv[4];
    st_ctx *ctx;
    const void *xyz[3];
    int32_t types[3];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    {
        uint32_t *idx = (uint32_t *)ta_data(env, argv[3], napi_uint32_array, &ni);
        if (!idx) return NULL;
        for (int a = 0; a < 3; ++a) {
            napi_typedarray_type nt;
            napi_value ab;
            size_t len = 0, off = 0, es = 0;
            void *data;
            bool is_ta = false;
            if (napi_is_typedarray(env, argv[a], &is_ta) != napi_ok || !is_ta ||
                napi_get_typedarray_info(env, argv[a], &nt, &len, &data, &ab, &off) != napi_ok ||
                !(types[a] = ply_type_of(nt, &es))) {
                napi_throw_type_error(env, NULL, "splat-hip: expected the reference's TypedArray columns");
                return NULL;
            }
            if (len != ni) {
                napi_throw_range_error(env, NULL, "splat-hip: x/y/z/indices lengths differ");
                return NULL;
            }
            xyz[a] = data;
        }
        if (!get_ctx(env, &ctx)) return NULL;
        int rc = st_morton_order_t(ctx, xyz, types, idx, (uint64_t)ni);
        if (rc != ST_OK) return throw_st(env, rc);
    }
    return argv[3];
fail:
    return NULL;
}

static napi_value js_webp_lossless(napi_env env, napi_callback_info info) {
    size_t argc = 4, len = 0;
    napi_value argv[4], out;
    st_ctx *ctx;
    uint8_t *webp = NULL;
    uint64_t size = 0;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    {
        const uint8_t *rgba = (const uint8_t *)ta_data(env, argv[0], napi_uint8_array, &len);
        const int32_t w = (int32_t)num(env, argv[1]), h = (int32_t)num(env, argv[2]);
        const int32_t stride = argc > 3 ? (int32_t)num(env, argv[3]) : w * 4;
        if (!rgba) return NULL;
        if (w < 1 || h < 1 || stride < w * 4 || (uint64_t)stride * (uint64_t)(h - 1) + (uint64_t)w * 4 > len) {
            napi_throw_range_error(env, NULL, "splat-hip: rgba buffer smaller than width x height");
            return NULL;
        }
        if (!get_ctx(env, &ctx)) return NULL;
        int rc = st_webp_lossless(ctx, rgba, w, h, stride, &webp, &size);
        if (rc != ST_OK) return throw_st(env, rc);
        NAPI_OK(napi_create_buffer_copy(env, size, webp, NULL, &out));
        st_free(webp);
        return out;
    }
fail:
    st_free(webp);
    return NULL;
}

static napi_value js_sog_bundle(napi_env env, napi_callback_info info) {
    size_t argc = 6, nd = 0;
    napi_value argv[6], out, buf;
    uint32_t m = 0;
    uint64_t n = 0, used = 0, size = 0;
    float **cols = NULL;
    char **names = NULL;
    uint8_t *zip = NULL;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[0], &m, &n))) return NULL;
    if (!(names = str_list(env, argv[1], m))) goto fail;
    {
        const int32_t iters = (int32_t)num(env, argv[2]);
        double *draws = (double *)ta_data(env, argv[3], napi_float64_array, &nd);
        const uint16_t dos_time = (uint16_t)num(env, argv[4]), dos_date = (uint16_t)num(env, argv[5]);
        if (!draws) goto fail;
        if (!get_ctx(env, &ctx)) goto fail;
        st_table tab = {n, (int32_t)m, (const char *const *)names, cols};
        int rc = st_sog_bundle(ctx, &tab, iters, draws, nd, &used, dos_time, dos_date, &zip, &size);
        if (rc != ST_OK) {
            free(cols);
            free_strs(names, m);
            return throw_st(env, rc);
        }
        NAPI_OK(napi_create_buffer_copy(env, size, zip, NULL, &buf));
        NAPI_OK(napi_create_object(env, &out));
        set_named(env, out, "archive", buf);
        set_named(env, out, "used", make_num(env, (double)used));
    }
    st_free(zip);
    free(cols);
    free_strs(names, m);
    return out;
fail:
    st_free(zip);
    free(cols);
    free_strs(names, m);
    return NULL;
}

/* sogFile(fd, cols, names, iters, draws: Float64Array, dosTime, dosDate) -> {used, size}: writeSog
 * into the open file fd (st_sog_file: the archive streamed while the SH k-means runs) */
static napi_value js_sog_file(napi_env env, napi_callback_info info) {
    size_t argc = 7, nd = 0;
    napi_value argv[7], out;
    uint32_t m = 0;
    uint64_t n = 0, used = 0, size = 0;
    float **cols = NULL;
    char **names = NULL;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(cols = f32_list(env, argv[1], &m, &n))) return NULL;
    if (!(names = str_list(env, argv[2], m))) goto fail;
    {
        const int32_t fd = (int32_t)num(env, argv[0]), iters = (int32_t)num(env, argv[3]);
        double *draws = (double *)ta_data(env, argv[4], napi_float64_array, &nd);
        const uint16_t dos_time = (uint16_t)num(env, argv[5]), dos_date = (uint16_t)num(env, argv[6]);
        if (!draws) goto fail;
        if (!get_ctx(env, &ctx)) goto fail;
        st_table tab = {n, (int32_t)m, (const char *const *)names, cols};
        const double t0 = now_ms();
        int rc = st_sog_file(ctx, &tab, iters, draws, nd, &used, fd, dos_time, dos_date, &size);
        if (getenv("ST_DEBUG")) fprintf(stderr, "[addon] sogFile: st_sog_file %.1f ms\n", now_ms() - t0);
        free(cols);
        free_strs(names, m);
        if (rc != ST_OK) return throw_st(env, rc);
        NAPI_OK(napi_create_object(env, &out));
        set_named(env, out, "used", make_num(env, (double)used));
        set_named(env, out, "size", make_num(env, (double)size));
        return out;
    }
fail:
    free(cols);
    free_strs(names, m);
    return NULL;
}

/* readPly(fd) -> {comments, elements: [{name, columns: [{name, data, lazy}]}]}.  By default the
 * values stay in HBM (st_ply_read_resident): `data` is allocated but unfilled, `lazy` is true, and
 * js/index.js hands it out only through materialize(); ST_READ_RESIDENT=0 fills every column
 * here (st_ply_read). */
static napi_value js_read_ply(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], out, els, comments;
    st_ctx *ctx;
    st_ply_header *h = NULL;
    const char *rm = getenv("ST_READ_RESIDENT");
    const int lazy = !(rm && strcmp(rm, "0") == 0);
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    {
        const int32_t fd = (int32_t)num(env, argv[0]);
        static const napi_typedarray_type tt[9] = {napi_uint8_array, napi_int8_array, napi_uint8_array,
                                                   napi_int16_array, napi_uint16_array, napi_int32_array,
                                                   napi_uint32_array, napi_float32_array, napi_float64_array};
        static const size_t ts[9] = {1, 1, 1, 2, 2, 4, 4, 4, 8};
        h = (st_ply_header *)calloc(1, sizeof *h);
        if (!h) goto fail;
        int rc = st_ply_read_header(fd, h);
        if (rc != ST_OK) {
            free(h);
            return throw_st(env, rc);
        }
        if (!get_ctx(env, &ctx)) goto fail;
        NAPI_OK(napi_create_object(env, &out));
        NAPI_OK(napi_create_array_with_length(env, (size_t)h->ncomments, &comments));
        {
            const char *c = h->comments;
            for (int32_t i = 0; i < h->ncomments; ++i) {
                const char *e = strchr(c, '\n');
                const size_t len = e ? (size_t)(e - c) : strlen(c);
                napi_value sv;
                napi_create_string_utf8(env, c, len, &sv);
                napi_set_element(env, comments, (uint32_t)i, sv);
                c = e ? e + 1 : c + len;
            }
        }
        NAPI_OK(napi_create_array_with_length(env, (size_t)h->nelements, &els));
        double t_alloc = 0, t_read = 0;
        for (int32_t ei = 0; ei < h->nelements; ++ei) {
            const double t0 = now_ms();
            const st_ply_element *el = &h->elements[ei];
            napi_value eo, cols, nm;
            void *ptrs[ST_PLY_MAX_PROPS];
            napi_create_object(env, &eo);
            napi_create_string_utf8(env, el->name, NAPI_AUTO_LENGTH, &nm);
            set_named(env, eo, "name", nm);
            napi_create_array_with_length(env, (size_t)el->nprops, &cols);
            for (int32_t p = 0; p < el->nprops; ++p) {
                napi_value co, pn, lz,
                    ta = lazy ? new_typed_ext(env, tt[el->props[p].type], (size_t)el->count, ts[el->props[p].type], &ptrs[p])
                              : new_typed_big(env, tt[el->props[p].type], (size_t)el->count, ts[el->props[p].type], &ptrs[p]);
                if (!ta) goto fail;
                napi_create_object(env, &co);
                napi_create_string_utf8(env, el->props[p].name, NAPI_AUTO_LENGTH, &pn);
                set_named(env, co, "name", pn);
                set_named(env, co, "data", ta);
                napi_get_boolean(env, lazy && el->count > 0, &lz);
                set_named(env, co, "lazy", lz);
                napi_set_element(env, cols, (uint32_t)p, co);
            }
            const double t1 = now_ms();
            rc = lazy ? st_ply_read_resident(ctx, fd, h, ei, ptrs) : st_ply_read(ctx, fd, h, ei, ptrs);
            t_alloc += t1 - t0;
            t_read += now_ms() - t1;
            if (rc != ST_OK) {
                free(h);
                return throw_st(env, rc);
            }
            set_named(env, eo, "columns", cols);
            napi_set_element(env, els, (uint32_t)ei, eo);
        }
        if (getenv("ST_DEBUG"))
            fprintf(stderr, "[addon] readPly: column arrays %.1f ms, st_ply_read %.1f ms\n", t_alloc, t_read);
        set_named(env, out, "comments", comments);
        set_named(env, out, "elements", els);
    }
    free(h);
    return out;
fail:
    free(h);
    return NULL;
}

/* materialize(typedArray): a resident readPly column's values copied down from HBM (st_ply_materialize;
 * no-op for any other array) */
static napi_value js_materialize(napi_env env, napi_callback_info info) {
    size_t argc = 1, length = 0, off = 0;
    napi_value argv[1], ab;
    bool is_ta = false;
    napi_typedarray_type type;
    void *data = NULL;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 1 || napi_is_typedarray(env, argv[0], &is_ta) != napi_ok || !is_ta ||
        napi_get_typedarray_info(env, argv[0], &type, &length, &data, &ab, &off) != napi_ok) {
        napi_throw_type_error(env, NULL, "splat-hip: materialize takes a TypedArray");
        return NULL;
    }
    if (!get_ctx(env, &ctx)) return NULL;
    {
        const int rc = st_ply_materialize(ctx, data);
        if (rc != ST_OK) return throw_st(env, rc);
    }
    return argv[0];
fail:
    return NULL;
}

/* array of TypedArrays of one type -> data pointers; n = common length */
static void **ta_list(napi_env env, napi_value arr, napi_typedarray_type want, uint32_t expect, uint64_t *n) {
    uint32_t m = 0;
    if (napi_get_array_length(env, arr, &m) != napi_ok || (expect && m != expect)) {
        napi_throw_type_error(env, NULL, "splat-hip: wrong column list");
        return NULL;
    }
    void **p = (void **)calloc(m ? m : 1, sizeof(void *));
    for (uint32_t i = 0; i < m; ++i) {
        napi_value e;
        size_t len = 0;
        napi_get_element(env, arr, i, &e);
        p[i] = ta_data(env, e, want, &len);
        if (!p[i]) {
            free(p);
            return NULL;
        }
        if (n) *n = len;
    }
    return p;
}

static napi_value js_decompress_ply(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], out;
    void **chunk = NULL, **vertex = NULL, **sh = NULL;
    uint64_t nch = 0, n = 0, nsv = 0;
    uint32_t nsh = 0;
    st_ctx *ctx;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!(chunk = ta_list(env, argv[0], napi_float32_array, 18, &nch))) goto fail;
    if (!(vertex = ta_list(env, argv[1], napi_uint32_array, 4, &n))) goto fail;
    NAPI_OK(napi_get_array_length(env, argv[2], &nsh));
    if (!(sh = ta_list(env, argv[2], napi_uint8_array, 0, &nsv))) goto fail;
    if (nch != (n + 255) / 256 || (nsh && nsv != n)) {
        napi_throw_range_error(env, NULL, "splat-hip: chunk/vertex/sh lengths do not match");
        goto fail;
    }
    {
        float *o[14 + 45];
        napi_value tv[14 + 45];
        if (nsh > 45) {
            napi_throw_range_error(env, NULL, "splat-hip: at most 45 SH columns");
            goto fail;
        }
        NAPI_OK(napi_create_array_with_length(env, 14 + nsh, &out));
        for (uint32_t k = 0; k < 14 + nsh; ++k) {
            void *d;
            tv[k] = new_typed(env, napi_float32_array, (size_t)n, 4, &d);
            o[k] = (float *)d;
            napi_set_element(env, out, k, tv[k]);
        }
        if (!get_ctx(env, &ctx)) goto fail;
        int rc = st_decompress_ply(ctx, n, (const float *const *)chunk, (const uint32_t *const *)vertex,
                                   (const uint8_t *const *)sh, (int32_t)nsh, o);
        if (rc != ST_OK) {
            free(chunk);
            free(vertex);
            free(sh);
            return throw_st(env, rc);
        }
    }
    free(chunk);
    free(vertex);
    free(sh);
    return out;
fail:
    free(chunk);
    free(vertex);
    free(sh);
    return NULL;
}

static napi_value init(napi_env env, napi_value exports) {
    static const struct {
        const char *name;
        napi_callback fn;
    } fns[] = {{"version", js_version},
               {"deviceCount", js_device_count},
               {"rcclInfo", js_rccl_info},
               {"lastHostReuse", js_last_host_reuse},
               {"quatFromEuler", js_quat_from_euler},
               {"transform", js_transform},
               {"filterFinite", js_filter_finite},
               {"filterNaN", js_filter_nan},
               {"setDevices", js_set_devices},
               {"getDevices", js_get_devices},
               {"combineLayout", js_combine_layout},
               {"mortonOrder", js_morton},
               {"packCompressed", js_pack_compressed},
               {"kmeans", js_kmeans},
               {"cluster1d", js_cluster1d},
               {"sog", js_sog},
               {"webpLossless", js_webp_lossless},
               {"sogBundle", js_sog_bundle},
               {"sogFile", js_sog_file},
               {"readPly", js_read_ply},
               {"materialize", js_materialize},
               {"decompressPly", js_decompress_ply},
               {"compressedPly", js_compressed_ply},
               {"compressedPlyFromFile", js_compressed_ply_file},
               {"compressedPlyToFile", js_compressed_ply_to_file},
               {"compressedPlyTableToFile", js_compressed_ply_table_to_file},
               {"sogBundleFromFile", js_sog_bundle_file},
               {"process", js_process},
               {"sogProcess", js_sog_process},
               {"sogBundleProcess", js_sog_bundle_process},
               {"transformTyped", js_transform_typed},
               {"mortonOrderTyped", js_morton_typed}};
    for (size_t i = 0; i < sizeof fns / sizeof fns[0]; ++i) {
        napi_value f;
        if (napi_create_function(env, fns[i].name, NAPI_AUTO_LENGTH, fns[i].fn, NULL, &f) != napi_ok) return NULL;
        napi_set_named_property(env, exports, fns[i].name, f);
    }
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
