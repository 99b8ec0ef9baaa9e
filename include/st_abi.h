/*
 * st_abi.h -- C-ABI of the MI355X splat-transform hot path (libsplat_hip.so).
 *
 * Plain pointers and sizes only.  Each entry point replaces one reference seam
 * (file:line into praveenpenumaka/splat-transform src/):
 *
 *   st_transform / st_dev_transform         transform(dataTable, t, r, s)      transform.ts:12-65
 *   st_quat_from_euler                      Quat.setFromEulerAngles             process.ts:75-79
 *   st_transform_params_make                Mat4.setTRS + Mat3.setFromQuat +
 *                                           new RotateSH(mat3)                  transform.ts:13-15,
 *                                                                               rotate-sh.ts:49-149
 *   st_filter_finite / st_dev_filter_finite filter(dt, isFinite-all) indices    process.ts:47-61,84-95
 *   st_filter_nan                           filterNaN: filter + permuteRows     process.ts:84-95
 *   st_dev_permute_rows[_t]                 DataTable.permuteRows               data-table.ts:135-149
 *   st_combine_layout / st_dev_combine      combine()                           index.ts:158-210
 *   st_dev_concat_rows                      combine() of float32 tables         index.ts:158-210
 *   st_morton_order / st_dev_morton_order   generateOrdering(dataTable, idx)    ordering.ts:4-110
 *   st_pack_compressed / st_dev_...         writeCompressedPly chunk loop +
 *                                           CompressedChunk.pack                write-compressed-ply.ts:56-109,
 *                                                                               compressed-chunk.ts:44-180
 *   st_kmeans / st_dev_kmeans               kmeans(points, k, iters) --no-gpu   k-means.ts:137-201,
 *                                                                               kd-tree.ts:9-100
 *   st_cluster1d / st_dev_cluster1d         cluster1d(dataTable, iters)         write-sog.ts:56-99
 *   st_sog / st_dev_sog                     writeSog texture + meta generation  write-sog.ts:110-370
 *   st_set_devices / st_group_sog /         writeSog with the rows sharded over
 *   st_dev_sog_sharded                      GPUs (RCCL; device choice of        write-sog.ts:241-243,313
 *                                           the reference's clusterer)
 *   st_dev_kmeans_* (step API)              one k-means iteration split at the
 *                                           centroid-sum exchange (multi-GPU)   k-means.ts:164-192
 *   st_dev_cluster1d_codebook               cluster1d's sorted codebook + byte
 *                                           labels                              write-sog.ts:69-88
 *   st_dev_sog_scatter / _shn_centroids     one shard's texels of writeSog      write-sog.ts:142-239,
 *                                                                               :319-348
 *   st_webp_lossless / st_dev_webp_lossless WebPEncodeLosslessRGBA (libwebp)   lib/webp_encode.c:19-29,
 *                                                                               utils/webp.ts:19-41
 *   st_dev_crc32                            Crc.update / value                  serialize/crc.ts:1-28
 *   st_zip_store                            ZipWriter (store, descriptors)      serialize/zip-writer.ts:35-135
 *   st_sog_meta_json                        JSON.stringify(meta)                write-sog.ts:271-293,350-361
 *   st_sog_bundle / st_dev_sog_bundle       writeSog to a .sog bundle           write-sog.ts:110-140,361-366
 *   st_ply_read_header / _parse_header      readPly header search + parseHeader readers/read-ply.ts:54-137
 *   st_ply_read / st_dev_ply_read           readPly element rows -> columns     read-ply.ts:139-188
 *   st_ply_read_resident (+ _materialize,   readPly, the values left in HBM     read-ply.ts:111-191
 *     _forget)                              until the host asks for them
 *   st_dev_ply_transpose                    (the same, rows already in HBM)     read-ply.ts:165-182
 *   st_decompress_ply / st_dev_...          decompressPly                       readers/decompress-ply.ts:82-232
 *   st_process                              processDataTable(dataTable, actions) process.ts:64-145
 *   st_ply_compressed_ply / st_ply_sog_bundle  readPly + processDataTable + writer, resident
 *                                           (the CLI's one-input path)           index.ts:463-496
 *   st_ply_compressed_ply_file /            the same + the output file written   write-compressed-ply.ts:31-115,
 *   st_compressed_ply_file                  at offsets as it leaves HBM          index.ts:101-154
 *   st_compressed_ply / st_dev_...          processDataTable + writeCompressedPly
 *                                           (CLI: in.ply [actions] out.compressed.ply) index.ts:463-496,
 *                                                                               write-compressed-ply.ts:31-115
 *
 * Conventions
 *  - Columns are SoA float32 arrays of n rows (the reference's Float32Array
 *    columns, read-ply.ts:148-150).  st_* entry points take HOST pointers and
 *    copy through HBM; st_dev_* take DEVICE pointers and run on the context's
 *    stream (asynchronously unless the function must return a count).
 *  - Math.random: k-means draws are supplied by the caller as a buffer of
 *    doubles in [0,1) in the order the reference consumes them; `used`
 *    returns how many were consumed.  ST_ERR_DRAWS if the buffer is short.
 *  - Every function returns ST_OK (0) or a negative st_status; the message is
 *    available from st_last_error() (thread-local).  Data anomalies that the
 *    reference tolerates (NaN quantises to 0, degenerate extents skip the
 *    Morton sort) are not errors.  Inputs that crash the reference's k-means
 *    (non-finite points) return ST_ERR_NONFINITE.
 */
#ifndef ST_ABI_H
#define ST_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ST_ABI_VERSION 1

enum st_status {
    ST_OK = 0,
    ST_ERR_ARG = -1,
    ST_ERR_HIP = -2,
    ST_ERR_NONFINITE = -3,
    ST_ERR_DRAWS = -4,
    ST_ERR_NOMEM = -5,
    ST_ERR_UNSUPPORTED = -6,
    ST_ERR_INTERNAL = -7
};

typedef struct st_ctx st_ctx;

/* SoA table of float32 columns (borrowed for the duration of a call). */
typedef struct {
    uint64_t n;                 /* rows */
    int32_t ncol;               /* columns */
    const char *const *names;   /* PLY property names: x y z f_dc_0 f_rest_k opacity scale_i rot_i ... */
    float *const *cols;         /* column base pointers (host or device, per entry point) */
} st_table;

/* Host-side constants of one transform() call: Mat4.setTRS (f32 storage),
 * the quaternion r, the uniform scale s and the RotateSH band matrices
 * (row-major, f64) built from Mat3.setFromQuat(r). */
typedef struct {
    float m4[16];
    double r[4]; /* x, y, z, w */
    double s;
    double sh1[9];
    double sh2[25];
    double sh3[49];
} st_transform_params;

typedef struct {
    int32_t width, height;          /* means/quats/scales/sh0/shN_labels textures (RGBA8) */
    double means_min[3], means_max[3];
    float scales_codebook[256];
    float sh0_codebook[256];
    int32_t sh_bands;               /* 0..3 */
    int32_t palette_size;           /* shN.count */
    float shn_codebook[256];
    int32_t shn_width, shn_height;  /* shN_centroids texture */
} st_sog_meta;

/* PLY header (readers/read-ply.ts:7-26); property types of read-ply.ts:28-40 */
enum st_ply_type {
    ST_PLY_CHAR = 1, ST_PLY_UCHAR, ST_PLY_SHORT, ST_PLY_USHORT, ST_PLY_INT, ST_PLY_UINT, ST_PLY_FLOAT, ST_PLY_DOUBLE
};
#define ST_PLY_MAX_ELEMENTS 16
#define ST_PLY_MAX_PROPS 256
#define ST_PLY_NAME 64
typedef struct {
    char name[ST_PLY_NAME];
    int32_t type; /* st_ply_type */
} st_ply_property;
typedef struct {
    char name[ST_PLY_NAME];
    uint64_t count;
    int32_t nprops;
    st_ply_property props[ST_PLY_MAX_PROPS];
} st_ply_element;
typedef struct {
    uint64_t header_bytes;   /* bytes up to and including "\nend_header\n" */
    int32_t nelements;
    int32_t ncomments;
    char comments[8192];     /* the comment texts, '\n'-separated */
    st_ply_element elements[ST_PLY_MAX_ELEMENTS];
} st_ply_header;

/* Typed SoA table: the reference's eight column types (data-table.ts:1-27) as st_ply_type
 * codes (ST_PLY_CHAR = Int8Array ... ST_PLY_FLOAT = Float32Array, ST_PLY_DOUBLE =
 * Float64Array).  Used where the reference handles every type: filterNaN, permuteRows,
 * combine.  Column data must be aligned to its element size. */
typedef struct {
    uint64_t n;
    int32_t ncol;
    const char *const *names;
    const int32_t *types;       /* st_ply_type per column */
    void *const *cols;
} st_ttable;

typedef struct {
    uint8_t *means_l, *means_u, *quats, *scales, *sh0; /* width*height*4 each */
    uint8_t *shn_centroids;                           /* shn_width*shn_height*4 (NULL if sh_bands==0) */
    uint8_t *shn_labels;                              /* width*height*4 (NULL if sh_bands==0) */
} st_sog_textures;

/* ---- runtime ------------------------------------------------------------ */
int st_abi_version(void);
const char *st_last_error(void);
int st_device_count(int32_t *count);
int st_ctx_create(int32_t device, st_ctx **out);
void st_ctx_destroy(st_ctx *ctx);
/* Run on a caller-owned hipStream_t (e.g. torch.cuda.current_stream()); NULL restores the context's own stream. */
int st_ctx_set_stream(st_ctx *ctx, void *hip_stream);
int st_ctx_synchronize(st_ctx *ctx);
/* Per-stage device timing (hipEvents) of the last st_*sog / st_*kmeans call, JSON text. */
const char *st_ctx_last_timings(st_ctx *ctx);
/* the last N-D k-means' assign classification on ctx, summed over its iterations, as JSON:
 * {"assigns", "points", "pairs" (two tile-halves settled by the exact fix-up), "ambiguous"
 * (the second sweep's candidate lists), "overflow" (first lists past 64 rows, collected again),
 * "walked_overflow" (past 2,048 rows too: the KdTree walk), "ties" (exact ties walked)}; "{}"
 * before the first.  Owned by ctx, valid until its next N-D k-means.  (No reference counterpart:
 * diagnostics of this build's exact assign.) */
const char *st_ctx_last_kmeans_stats(st_ctx *ctx);
/* The writeSog host forms (st_sog, st_sog_bundle, st_sog_file) run on the device columns the
 * last st_ply_read left resident when the caller's table is that read's host columns, unchanged:
 * the step starts at once on them while host threads compare every byte of the host columns
 * with the read's pinned copy; the first changed byte abandons the run (nothing has left the
 * device), and the call uploads the columns and runs again.  This reports, for the last such
 * call on ctx, how many columns / bytes ran from the resident copy (0 / 0: uploaded).
 * ST_HOST_MIRROR=0 disables the reuse.  (No reference counterpart: the reference's readPly ->
 * writeSog keeps the table in JS memory, index.ts:433-510.) */
int st_ctx_last_host_reuse(st_ctx *ctx, uint64_t *columns, uint64_t *bytes);
/* Kernel profiling: when enabled, the library brackets its named hot kernels
 * ("kn.sweep", "mo.sort", ...) with hipEvents on the context stream; stats
 * accumulate until st_ctx_reset_kernel_stats.  Query after a synchronize. */
int st_ctx_set_profiling(st_ctx *ctx, int32_t enable);
int st_ctx_reset_kernel_stats(st_ctx *ctx);
int st_ctx_kernel_stats(st_ctx *ctx, const char *name, double *total_ms, uint64_t *launches);
/* Output verification (bench.py, tests): when enabled, every N-D k-means (d > 1) keeps a
 * device copy of the centroids its LAST assign used, its final centroids and its labels
 * (k-means.ts:164-192: the returned labels come from the last assign, the centroids from the
 * update after it).  st_ctx_verify_snapshot writes d, k, n and, where the pointers are not
 * NULL, copies them into caller DEVICE buffers on the context stream: centroids [d][k]
 * float32, labels uint32[n].  Costs three device copies per k-means call while enabled. */
int st_ctx_set_verify(st_ctx *ctx, int32_t enable);
int st_ctx_verify_snapshot(st_ctx *ctx, float *prev_centroids, float *centroids, uint32_t *labels,
                           int32_t *d, int32_t *k, uint64_t *n);

/* ---- host constants ------------------------------------------------------ */
int st_quat_from_euler(double ex_deg, double ey_deg, double ez_deg, double q_xyzw[4]);
int st_transform_params_make(const double t[3], const double r_xyzw[4], double s, st_transform_params *out);
/* SOG texture geometry (write-sog.ts:117-118, :310, :319) */
int st_sog_geometry(uint64_t n, int32_t sh_coeffs, int32_t *width, int32_t *height,
                    int32_t *palette_size, int32_t *shn_width, int32_t *shn_height);

/* ---- host-memory entry points ---------------------------------------------- */
int st_transform(st_ctx *ctx, const st_table *table, const st_transform_params *p);
int st_filter_finite(st_ctx *ctx, const st_table *table, uint32_t *out_idx, uint64_t *out_n);
/* filterNaN on host columns in one call (process.ts:84-95 -> filter -> permuteRows): the table
 * is uploaded once, the surviving rows are compacted on the device and the first *out_m rows of
 * each dst column (host, src's types, capacity n rows) receive them */
int st_filter_nan(st_ctx *ctx, const st_ttable *src, const st_ttable *dst, uint64_t *out_m);
int st_morton_order(st_ctx *ctx, const float *x, const float *y, const float *z, uint32_t *indices, uint64_t n);
int st_pack_compressed(st_ctx *ctx, const st_table *table, const uint32_t *order,
                       float *chunk, uint32_t *vertex, uint8_t *sh);
int st_kmeans(st_ctx *ctx, const float *const *cols, int32_t d, uint64_t n, int32_t k, int32_t iters,
              const double *draws, uint64_t ndraws, uint64_t *used, float *centroids, uint32_t *labels);
int st_cluster1d(st_ctx *ctx, const float *const *cols, int32_t ncols, uint64_t n, int32_t iters,
                 const double *draws, uint64_t ndraws, uint64_t *used, float *centroids256, uint8_t *labels);
int st_sog(st_ctx *ctx, const st_table *table, int32_t iters, const double *draws, uint64_t ndraws,
           uint64_t *used, st_sog_meta *meta, const st_sog_textures *out);

/* ---- device-memory entry points (device pointers, context stream) ---------- */
int st_dev_transform(st_ctx *ctx, const st_table *table, const st_transform_params *p);
int st_dev_filter_finite(st_ctx *ctx, const st_table *table, uint32_t *out_idx, uint64_t *out_n);
int st_dev_permute_rows(st_ctx *ctx, const st_table *src, const uint32_t *idx, uint64_t m, const st_table *dst);
int st_dev_concat_rows(st_ctx *ctx, const st_table *const *srcs, int32_t nsrc, const st_table *dst);
/* typed forms (every column type, as the reference):
 *   filterNaN's indices: float32 and float64 columns are tested with isFinite, integer
 *     columns are always finite (process.ts:84-95)
 *   permuteRows: dst[c][j] = src[c][idx[j]], dst columns of src's types (data-table.ts:135-149)
 *   combine: st_combine_layout lists the result columns -- (table, column) of each, the
 *     first table's columns then every later column without a (name, type) match
 *     (index.ts:164-178); st_dev_combine fills a dst of that layout with sum(n) rows: zeros,
 *     then each source column at its table's row offset in its first (name, type) match */
int st_dev_filter_finite_t(st_ctx *ctx, const st_ttable *table, uint32_t *out_idx, uint64_t *out_n);
int st_dev_permute_rows_t(st_ctx *ctx, const st_ttable *src, const uint32_t *idx, uint64_t m, const st_ttable *dst);
/* host only (no device); col_table / col_index may be NULL to query the count */
int st_combine_layout(const st_ttable *const *srcs, int32_t nsrc, int32_t *col_table, int32_t *col_index,
                      int32_t *ncol);
int st_dev_combine(st_ctx *ctx, const st_ttable *const *srcs, int32_t nsrc, const st_ttable *dst);
int st_dev_morton_order(st_ctx *ctx, const float *x, const float *y, const float *z, uint32_t *indices, uint64_t n);
int st_dev_pack_compressed(st_ctx *ctx, const st_table *table, const uint32_t *order,
                           float *chunk, uint32_t *vertex, uint8_t *sh);
/* draws stay on the host (the reference's Math.random lives there) */
int st_dev_kmeans(st_ctx *ctx, const float *const *cols, int32_t d, uint64_t n, int32_t k, int32_t iters,
                  const double *draws, uint64_t ndraws, uint64_t *used, float *centroids, uint32_t *labels);
int st_dev_cluster1d(st_ctx *ctx, const float *const *cols, int32_t ncols, uint64_t n, int32_t iters,
                     const double *draws, uint64_t ndraws, uint64_t *used, float *centroids256, uint8_t *labels);
int st_dev_sog(st_ctx *ctx, const st_table *table, int32_t iters, const double *draws, uint64_t ndraws,
               uint64_t *used, st_sog_meta *meta, const st_sog_textures *out);

/* ---- processDataTable + writeCompressedPly in one upload (BASELINE config 3) -----
 * The reference's action list (process.ts:64-145) applied to a typed table in order:
 *   ST_ACTION_TRANSFORM     one transform() pass (translate / rotate / scale, process.ts:72-83),
 *                           params from st_transform_params_make; columns of any type (as
 *                           st_transform_t)
 *   ST_ACTION_FILTER_NAN    filterNaN (process.ts:84-95)
 *   ST_ACTION_FILTER_VALUE  filterByValue (process.ts:97-109): row[column] <compare> value;
 *                           compare outside ST_CMP_LT..ST_CMP_NEQ keeps every row (:108)
 *   ST_ACTION_FILTER_BANDS  filterBands (process.ts:110-134): f_rest columns renamed / dropped
 *                           (the input band is read from the ORIGINAL table, as :111 does)
 *   ST_ACTION_PARAM         no-op (:135-138)
 * st_process: the processed table's columns are matched by (name, type) into dst (host, capacity
 * src->n rows); *out_m = its rows.  st_compressed_ply: the processed table goes on through
 * writeCompressedPly's ordering and chunk loop (write-compressed-ply.ts:31-115): chunk
 * ceil(m/256)*18 f32, vertex m*4 u32, sh m*3C u8 (host, sized for src->n rows and src's band);
 * *out_m = m, *out_sh_coeffs = C.  st_dev_compressed_ply: the same over device columns
 * (transformed in place, like the reference's table) into device outputs. */
enum st_action_kind {
    ST_ACTION_TRANSFORM = 1, ST_ACTION_FILTER_NAN, ST_ACTION_FILTER_VALUE, ST_ACTION_FILTER_BANDS, ST_ACTION_PARAM
};
enum st_compare { ST_CMP_LT = 0, ST_CMP_LTE, ST_CMP_GT, ST_CMP_GTE, ST_CMP_EQ, ST_CMP_NEQ };
typedef struct {
    int32_t kind;                    /* st_action_kind */
    int32_t compare;                 /* ST_ACTION_FILTER_VALUE: st_compare */
    const char *column;              /* ST_ACTION_FILTER_VALUE */
    double value;                    /* ST_ACTION_FILTER_VALUE */
    int32_t bands;                   /* ST_ACTION_FILTER_BANDS: output bands 0..3 */
    st_transform_params transform;   /* ST_ACTION_TRANSFORM */
} st_action;
int st_process(st_ctx *ctx, const st_ttable *src, const st_action *actions, int32_t nactions, const st_ttable *dst,
               uint64_t *out_m);
int st_compressed_ply(st_ctx *ctx, const st_ttable *src, const st_action *actions, int32_t nactions, float *chunk,
                      uint32_t *vertex, uint8_t *sh, uint64_t *out_m, int32_t *out_sh_coeffs);
int st_dev_compressed_ply(st_ctx *ctx, const st_ttable *src, const st_action *actions, int32_t nactions,
                          float *chunk, uint32_t *vertex, uint8_t *sh, uint64_t *out_m, int32_t *out_sh_coeffs);
/* The same straight from the PLY file (`in.ply [actions] out.compressed.ply` / `in.ply [actions]
 * out.sog`, index.ts:463-496): the element's rows stream page cache -> pinned -> HBM
 * (st_dev_ply_read, read-ply.ts:139-188) and stay resident through the actions and the writer;
 * only the outputs cross back.  element < 0 selects the element named "vertex".
 * st_ply_compressed_ply: outputs sized for the element's row count and band.
 * st_ply_sog_bundle: st_sog_bundle of the processed table (malloc'd archive, st_free); with
 * st_set_devices(n > 1) the processed columns are sharded over the group from the host. */
int st_ply_compressed_ply(st_ctx *ctx, int32_t fd, const st_ply_header *h, int32_t element, const st_action *actions,
                          int32_t nactions, float *chunk, uint32_t *vertex, uint8_t *sh, uint64_t *out_m,
                          int32_t *out_sh_coeffs);
/* writeCompressedPly into a file (write-compressed-ply.ts:31-115 and the CLI's write of the
 * output, index.ts:101-154): st_ply_compressed_ply / st_compressed_ply's chain, then the header
 * (the reference's text, "comment Generated by splat-transform <version>"; version NULL =
 * "0.10.1") and the chunk / vertex / sh arrays written to out_fd at offsets from its current
 * position (where the reference's FileHandle.write calls would go; the CLI's fresh output: 0)
 * as they come down from HBM through pinned slots (a host thread writes one slot while the next
 * one copies); the descriptor's position ends after the output and a longer file is cut there,
 * so a reused output needs no O_TRUNC.  out_fd must be a seekable descriptor open for writing
 * and not O_APPEND (ST_ERR_ARG before any work).  *size = the bytes written.
 * st_compressed_ply_file takes a host table (uploaded once). */
int st_ply_compressed_ply_file(st_ctx *ctx, int32_t fd, const st_ply_header *h, int32_t element,
                               const st_action *actions, int32_t nactions, int32_t out_fd, const char *version,
                               uint64_t *out_m, int32_t *out_sh_coeffs, uint64_t *size);
int st_compressed_ply_file(st_ctx *ctx, const st_ttable *src, const st_action *actions, int32_t nactions,
                           int32_t out_fd, const char *version, uint64_t *out_m, int32_t *out_sh_coeffs,
                           uint64_t *size);
int st_ply_sog_bundle(st_ctx *ctx, int32_t fd, const st_ply_header *h, int32_t element, const st_action *actions,
                      int32_t nactions, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                      uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *out_size);

/* ---- every column type on the writers' path ---------------------------------
 * The reference reads its columns through getRow (data-table.ts:63-68: each element as a JS
 * number, whatever the TypedArray) and writes through setRow (:70-76: a TypedArray store), so
 * a PLY with double (or integer) x / y / z / rot / scale / f_rest properties transforms, orders
 * and compresses.  These forms take typed tables (st_ttable, ST_PLY_* types):
 *   st_transform_t / st_dev_transform_t   transform() in place (transform.ts:12-65): f64
 *       arithmetic on the numbers, TypedArray stores (Float32 rounds, Float64 keeps, integers
 *       take ToInt32 cut to their width); SH through the Float32Array shCoeffs (transform.ts:21)
 *   st_morton_order_t / st_dev_morton_order_t   generateOrdering (ordering.ts:4-110) of x / y / z
 *       of any types (keys from the JS numbers)
 *   st_sog_process / st_sog_bundle_process   processDataTable (the actions, as st_process) then
 *       writeSog (write-sog.ts:110-370) of a typed host table: the textures + meta (as st_sog)
 *       or the .sog archive (as st_sog_bundle, malloc'd, st_free).  Positions, rotations and
 *       opacity are read as numbers; cluster1d and the k-means points through Float32Arrays;
 *       calcAverage (k-means.ts:41-63) sums the numbers.  With st_set_devices(n > 1) the
 *       processed columns must be float32 (the sharded path moves float32 columns)
 *   st_dev_sog_t   writeSog's device part over a typed device table
 * st_process / st_compressed_ply / st_dev_compressed_ply / st_ply_* take every type too
 * (transform actions, the writer's Morton order, chunk members and SH bytes). */
int st_transform_t(st_ctx *ctx, const st_ttable *table, const st_transform_params *p);
int st_dev_transform_t(st_ctx *ctx, const st_ttable *table, const st_transform_params *p);
int st_morton_order_t(st_ctx *ctx, const void *const xyz[3], const int32_t types[3], uint32_t *indices, uint64_t n);
int st_dev_morton_order_t(st_ctx *ctx, const void *const xyz[3], const int32_t types[3], uint32_t *indices,
                          uint64_t n);
int st_sog_process(st_ctx *ctx, const st_ttable *src, const st_action *actions, int32_t nactions, int32_t iters,
                   const double *draws, uint64_t ndraws, uint64_t *used, st_sog_meta *meta,
                   const st_sog_textures *out);
int st_sog_bundle_process(st_ctx *ctx, const st_ttable *src, const st_action *actions, int32_t nactions,
                          int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used, uint16_t dos_time,
                          uint16_t dos_date, uint8_t **out, uint64_t *out_size);
int st_dev_sog_t(st_ctx *ctx, const st_ttable *table, int32_t iters, const double *draws, uint64_t ndraws,
                 uint64_t *used, st_sog_meta *meta, const st_sog_textures *out);

/* ---- multi-GPU building blocks -----------------------------------
 * One process per GPU; rows are sharded in contiguous ranges in rank order; the
 * caller runs the collectives between calls (splat-transform_amd/py/splat_dist.py
 * composes them into kmeans / cluster1d / writeSog over the whole table).
 * k-means iteration = assign -> partials -> [allreduce sum/sum/min/sum] -> finish
 * -> [segment-ordered chain of seqsum for the pending pairs] -> average -> re-seed
 * empties from the draws (host).  Sums are [nseg][d][k] f64, counts [nseg][k];
 * a segment is a part of the shard that is contiguous in the global point order
 * (the shard for d > 1; one column of cluster1d's concatenation for d == 1). */
/* NaN-ignoring per-column min/max (+inf/-inf for a column without numbers) */
int st_dev_minmax(st_ctx *ctx, const float *const *cols, int32_t ncols, uint64_t n, double *lo, double *hi);
/* validates (ST_ERR_NONFINITE) and prepares the local point set for assign/partials */
int st_dev_kmeans_prepare(st_ctx *ctx, const float *const *cols, int32_t d, uint64_t n);
/* initializeCentroids (k-means.ts:8-20) over the global table of n rows, identical on every rank:
 * rows (device, k entries) = the first k distinct floor(draw * n) in draw order; *used = draws
 * consumed (replaces splat_dist's host selection; the owners then supply the rows) */
int st_dev_kmeans_init_rows(st_ctx *ctx, const double *draws, uint64_t ndraws, uint64_t n, int32_t k,
                            uint32_t *rows, uint64_t *used);
/* out[c * k + i] (device) = cols[c][rows[i] - offset] for the rows this rank holds
 * (offset <= rows[i] < offset + n_local), bit pattern 0 elsewhere: an integer SUM of the bit
 * patterns over the ranks assembles the global rows exactly (-0 and NaN payloads included) */
int st_dev_gather_rows(st_ctx *ctx, const float *const *cols, int32_t d, uint64_t n_local, uint64_t offset,
                       const uint32_t *rows, int32_t k, float *out);
/* exact nearest centroid (KdTree.findNearest semantics) of each local point */
int st_dev_kmeans_assign(st_ctx *ctx, const float *const *cols, int32_t d, uint64_t n, int32_t k,
                         const float *centroids, uint32_t *labels);
/* per (segment, dim, cluster): f64 sum in ascending point order, sum|x|, smallest ulp exponent; counts */
int st_dev_kmeans_partials(st_ctx *ctx, const float *const *cols, int32_t d, uint64_t n, int32_t nseg, int32_t k,
                           const uint32_t *labels, double *sums, double *sabs, int32_t *emin, uint32_t *counts);
/* continue running[i] (pair = cluster*d + dim) over this rank's members of segment seg, exactly as the
 * sequential f64 sum; emin / sabs are the global (reduced) partials [d][k] */
int st_dev_kmeans_seqsum(st_ctx *ctx, int32_t d, int32_t k, int32_t seg, const uint32_t *pairs, uint32_t npairs,
                         double *running, const int32_t *emin, const double *sabs);
/* global (reduced) partials -> centroids where the sum is certified exact; the rest listed in pending
 * (ascending pair order, *npending on the host); clusters with count 0 are left untouched */
int st_dev_kmeans_finish(st_ctx *ctx, int32_t d, int32_t k, const double *sums, const double *sabs,
                         const int32_t *emin, const uint32_t *counts, float *centroids, uint32_t *pending,
                         uint32_t *npending);
int st_dev_kmeans_average(st_ctx *ctx, int32_t d, int32_t k, const uint32_t *pairs, uint32_t npairs,
                          const double *running, const uint32_t *counts, float *centroids);
int st_dev_cluster1d_codebook(st_ctx *ctx, const float *centroids, const uint32_t *labels, uint64_t total,
                              float *codebook256, uint8_t *labels8);
/* writeSog texels of the local rows at their global sorted positions pos[i] (other texels untouched);
 * lo/hi: global NaN-ignoring x/y/z extents; label arrays per local row (NULL skips that texture);
 * fills meta->means_min/max */
int st_dev_sog_scatter(st_ctx *ctx, const st_table *local, const uint32_t *pos, const double lo[3], const double hi[3],
                       const uint8_t *scale_labels, const uint8_t *color_labels, const uint32_t *shn_labels,
                       st_sog_meta *meta, const st_sog_textures *out);
int st_dev_sog_shn_centroids(st_ctx *ctx, const uint8_t *codebook_labels, int32_t sh_coeffs, int32_t palette,
                             uint8_t *out);

/* ---- multi-GPU writeSog, native (SURVEY 8b st_set_devices, 8e) ----------------
 * The reference picks one device for its clusterer (write-sog.ts:241-243, :313); here the
 * splat rows are sharded across GPUs and the library runs the whole writeSog: k-means
 * centroid sums all-reduced over RCCL every iteration (exact: DESIGN.md (e)), rank 0 orders
 * the global table (Morton) and gathers the texels.  Results equal st_sog on the global table.
 * Rows of the global table = the input tables concatenated in order (combine(), index.ts:
 * 158-210: float32 columns by name, absent columns zero, band from the union of names). */
typedef struct st_comm st_comm;
typedef struct st_group st_group;
/* process-wide: st_sog / st_sog_bundle shard their rows over GPUs 0..ngpu-1 (one host thread
 * and stream per GPU, RCCL communicators from ncclCommInitAll); 1 (default) = one device */
int st_set_devices(int32_t ngpu);
int st_get_devices(int32_t *ngpu);
/* one process per GPU: rank 0 creates the id, the launcher distributes it, every rank joins */
int st_comm_unique_id(uint8_t id[128]);
int st_comm_init_rank(st_ctx *ctx, int32_t world, int32_t rank, const uint8_t id[128], st_comm **out);
/* the same job of one-rank processes with the bytes exchanged through host shared memory
 * instead of RCCL (several ranks on one GPU, which RCCL refuses: the process layout of the
 * N-GPU job rehearsed on one card).  Every rank passes the same `name` ([A-Za-z0-9_.-], unique
 * per job; rank 0 creates /dev/shm/st_<name>, which is unlinked once every rank has attached),
 * slot_bytes (per-rank staging slot, multiple of 4096; 0 = 32 MiB) and timeout_s (longest wait
 * for a peer before the job is aborted; <= 0 = 600 s).  The ranks must all attach within
 * timeout_s when it is set (> 0), within 120 s when it is not; the environment variable
 * ST_SHM_ATTACH_S overrides the attach wait.  A peer process that exits, or a rank that fails,
 * makes every rank's next exchange fail. */
int st_comm_init_host(st_ctx *ctx, int32_t world, int32_t rank, const char *name, uint64_t slot_bytes,
                      double timeout_s, st_comm **out);
void st_comm_destroy(st_comm *comm);
/* ranks in the communicator (ncclCommCount for RCCL): the bench reports it as `rccl_ranks` */
int st_comm_count(const st_comm *comm, int32_t *count);
/* the RCCL the library's collectives run on (loaded on first use, no GPU needed): its
 * ncclGetVersion (e.g. 22707 = 2.27.7) and the real path of the file.  Both hosts load the same
 * file by path -- /opt/rocm/lib/librccl.so.1 unless ST_RCCL names another, or ST_RCCL=process
 * (the copy of soname librccl.so.1 already in the process: torch's under Python) -- under a
 * handle of its own (RTLD_LOCAL).  path may be NULL.  ST_ERR_INTERNAL if it cannot be loaded. */
int st_rccl_info(int32_t *version, char *path, uint64_t path_len);
/* one rank's part of a sharded writeSog: `locals` are this rank's tables (device columns; its
 * files or file parts, in global order); every rank calls it with the same iters and draws.
 * meta / out (device textures) are written on rank 0 only. */
int st_dev_sog_sharded(st_ctx *ctx, st_comm *comm, const st_table *const *locals, int32_t nlocal, int32_t iters,
                       const double *draws, uint64_t ndraws, uint64_t *used, st_sog_meta *meta,
                       const st_sog_textures *out);
/* a set of ranks in this process: devices[r] is rank r's GPU (repeats allowed with
 * host_staged != 0: the exchange then goes through host memory -- several ranks on one GPU) */
int st_group_create(const int32_t *devices, int32_t n, int32_t host_staged, st_group **out);
void st_group_destroy(st_group *g);
/* writeSog of the concatenation of host tables; rank r takes global rows [splits[r], splits[r+1])
 * (splits: n + 1 ascending bounds from 0 to the row count; NULL = an even split); textures to
 * host memory (as st_sog) or the .sog archive (as st_sog_bundle) */
int st_group_sog(st_group *g, const st_table *const *tables, int32_t ntables, const uint64_t *splits, int32_t iters,
                 const double *draws, uint64_t ndraws, uint64_t *used, st_sog_meta *meta,
                 const st_sog_textures *out);
int st_group_sog_bundle(st_group *g, const st_table *const *tables, int32_t ntables, const uint64_t *splits,
                        int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used, uint16_t dos_time,
                        uint16_t dos_date, uint8_t **out, uint64_t *out_size);
/* the same with each input table's processDataTable actions (process.ts:64-145: the CLI's
 * `a.ply [actions] b.ply [actions] out.sog`) applied on the GPUs to each rank's part of that
 * input before writeSog: transform and the filters are row-local (the filtered
 * parts concatenate to the filtered input; the shard offsets come from the all-gathered survivor
 * counts); nactions[t] == 0 leaves table t as it is.  With one input its list may also carry the
 * output's actions (combine of one table is the table, index.ts:158-160). */
int st_group_sog_bundle_process(st_group *g, const st_table *const *tables, int32_t ntables, const uint64_t *splits,
                                const st_action *const *actions, const int32_t *nactions, int32_t iters,
                                const double *draws, uint64_t ndraws, uint64_t *used, uint16_t dos_time,
                                uint16_t dos_date, uint8_t **out, uint64_t *out_size);

/* ---- WebP lossless, CRC-32, the .sog container ---------------
 * WebP: a valid lossless VP8L stream (predictor transform + canonical prefix
 * codes) that decodes to exactly the input RGBA; parity is at the decoded-pixel
 * level, the bytes differ from libwebp's.  Images are 1..16384 on each side. */
/* worst-case .webp size for a width x height image (0 if out of range) */
uint64_t st_webp_max_size(int32_t width, int32_t height);
/* device RGBA8 (stride bytes per row, multiple of 4) -> device .webp bytes (cap >= st_webp_max_size) */
int st_dev_webp_lossless(st_ctx *ctx, const uint8_t *rgba, int32_t width, int32_t height, int32_t stride,
                         uint8_t *out, uint64_t cap, uint64_t *size);
/* host form of WebPEncodeLosslessRGBA: *out is malloc'd, release with st_free */
int st_webp_lossless(st_ctx *ctx, const uint8_t *rgba, int32_t width, int32_t height, int32_t stride,
                     uint8_t **out, uint64_t *size);
/* zlib-compatible CRC-32 of n device bytes, continuing from crc_in (0 = fresh; crc.ts value()) */
int st_dev_crc32(st_ctx *ctx, const uint8_t *data, uint64_t n, uint32_t crc_in, uint32_t *out);
/* host: the store-only ZIP of zip-writer.ts (entries in order, CRCs given); *out malloc'd */
int st_zip_store(const char *const *names, const uint8_t *const *data, const uint64_t *sizes,
                 const uint32_t *crcs, int32_t count, uint16_t dos_time, uint16_t dos_date,
                 uint8_t **out, uint64_t *out_size);
/* host: meta.json text of writeSog (JS number formatting); *out malloc'd, NUL-terminated */
int st_sog_meta_json(const st_sog_meta *meta, uint64_t count, char **out, uint64_t *out_size);
/* the .sog archive of textures resident on the device (st_dev_sog's outputs):
 * WebP encode + CRC on the device, ZIP layout on the host.  dos_time/dos_date are
 * the ZipWriter's clock fields (zip-writer.ts:39-41).  *out malloc'd (st_free). */
int st_dev_sog_bundle(st_ctx *ctx, const st_sog_meta *meta, uint64_t count, const st_sog_textures *tex,
                      uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *size);
/* as st_dev_sog_bundle, but *out borrows the context's pinned archive buffer (valid
 * until the next bundle call on ctx; no copy) -- what a writer hands to write(2) */
int st_dev_sog_bundle_view(st_ctx *ctx, const st_sog_meta *meta, uint64_t count, const st_sog_textures *tex,
                           uint16_t dos_time, uint16_t dos_date, const uint8_t **out, uint64_t *size);
/* writeSog into a file (write-sog.ts:110-370 and the CLI's write of the .sog, index.ts:101-154):
 * st_dev_sog with its archive streamed to the open file descriptor fd (written from offset 0) --
 * the five textures that are final before the SH palette k-means (means_l/u, quats, scales,
 * sh0) are WebP-encoded on a side context and written while the k-means runs, the shN
 * textures, meta.json and the central directory after it.  The file holds the same bytes as
 * st_dev_sog_bundle's archive and is cut to its length; *size = that length.  fd must be
 * seekable (a regular file opened for writing; the archive goes out with pwrite at absolute
 * offsets): a pipe or socket fails with ST_ERR_ARG before any work.  The caller opens and
 * closes fd; open it without O_TRUNC (the call cuts the file itself: on ext4 a file truncated to
 * zero and rewritten is flushed at close, and its old pages are freed at the open). */
int st_dev_sog_file(st_ctx *ctx, const st_table *table, int32_t iters, const double *draws, uint64_t ndraws,
                    uint64_t *used, st_sog_meta *meta, const st_sog_textures *out, int32_t fd, uint16_t dos_time,
                    uint16_t dos_date, uint64_t *size);
/* the same from a host table (uploaded; st_set_devices > 1: the group's archive written whole,
 * from offset 0, the file cut to its length; the same fd requirement) */
int st_sog_file(st_ctx *ctx, const st_table *table, int32_t iters, const double *draws, uint64_t ndraws,
                uint64_t *used, int32_t fd, uint16_t dos_time, uint16_t dos_date, uint64_t *size);
/* the whole writeSog(.sog) from a host table: st_sog + st_dev_sog_bundle */
int st_sog_bundle(st_ctx *ctx, const st_table *table, int32_t iters, const double *draws, uint64_t ndraws,
                  uint64_t *used, uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *size);
void st_free(void *p);

/* ---- PLY ingest and the compressed-PLY reader ----------------
 * Same header grammar and errors as readPly (binary little-endian bodies; the
 * "format" line is not checked, as in the reference).  A body shorter than the
 * header declares is an error here (the reference silently keeps stale bytes). */
int st_ply_parse_header(const uint8_t *data, uint64_t len, st_ply_header *out);
int st_ply_read_header(int32_t fd, st_ply_header *out);   /* pread of the first <= 128 KiB */
uint64_t st_ply_row_bytes(const st_ply_header *h, int32_t element);
/* element rows (row_bytes each, 4-byte aligned, device) -> per-property device columns */
int st_dev_ply_transpose(st_ctx *ctx, const st_ply_header *h, int32_t element, const uint8_t *rows,
                         uint64_t nrows, void *const *cols);
/* element `element` of the file fd -> device columns (pinned double-buffered chunks, H2D, transpose) */
int st_dev_ply_read(st_ctx *ctx, int32_t fd, const st_ply_header *h, int32_t element, void *const *cols);
/* the same into host columns (readPly's TypedArrays) */
int st_ply_read(st_ctx *ctx, int32_t fd, const st_ply_header *h, int32_t element, void *const *host_cols);
/* readPly with the values left in HBM (replaces read-ply.ts:111-191 for a host that defers the
 * host copy): element `element` goes to the device columns only, and host_cols are registered
 * as that element's lazy columns -- their memory is NOT written until st_ply_materialize.  The
 * writeSog host forms (st_sog, st_sog_bundle, st_sog_file) given a lazy column run on its device
 * copy directly; every other host form copies it down first.  Each lazy column holds a device
 * block of its own until it is materialized or st_ply_forget-ten (later reads do not touch it);
 * the caller keeps the host column alive until then. */
int st_ply_read_resident(st_ctx *ctx, int32_t fd, const st_ply_header *h, int32_t element, void *const *host_cols);
/* a lazy column's values copied into its host memory (then an ordinary host column: the caller
 * may change it); no-op for any other pointer */
int st_ply_materialize(st_ctx *ctx, const void *host_col);
/* drop the lazy or mirrored column at host_col without copying (its memory is being released) */
int st_ply_forget(st_ctx *ctx, const void *host_col);
/* decompressPly: chunk = the 18 float columns min_x..max_b in decompress-ply.ts:14-33 order,
 * vertex = packed_position, packed_rotation, packed_scale, packed_color; sh = nsh (0/9/24/45)
 * uint8 f_rest columns; out = x y z f_dc_0..2 opacity rot_0..3 scale_0..2 then f_rest_0.. */
int st_dev_decompress_ply(st_ctx *ctx, uint64_t n, const float *const *chunk, const uint32_t *const *vertex,
                          const uint8_t *const *sh, int32_t nsh, float *const *out);
int st_decompress_ply(st_ctx *ctx, uint64_t n, const float *const *chunk, const uint32_t *const *vertex,
                      const uint8_t *const *sh, int32_t nsh, float *const *out);

#ifdef __cplusplus
}
#endif
#endif /* ST_ABI_H */
