// st_internal.h -- shared runtime pieces of libsplat_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <functional>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/st_abi.h"

namespace st {

// ---------------------------------------------------------------------------
// errors: internal code throws st::Error, the extern "C" boundary converts it
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

// a host form that ran on st_ply_read's device twins of the caller's columns while the columns
// were compared with their pinned twins (st_host_api.hip: run_host_sog) stops with this when the
// compare finds a changed byte; the call then uploads the columns and runs again
struct SpecAbort : Error {
    SpecAbort() : Error(ST_ERR_INTERNAL, "speculative run abandoned: the host columns changed since st_ply_read") {}
};

#define ST_HIP(expr)                                                                          \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            throw ::st::Error(ST_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// ST_SYNC_CHECK=1 (read when a context is created): every launch check also synchronizes the
// device, so a kernel's fault is reported at the launch that caused it (debugging)
extern bool g_sync_check;
#define ST_LAUNCH_CHECK()                                       \
    do {                                                        \
        ST_HIP(hipGetLastError());                              \
        if (::st::g_sync_check) ST_HIP(hipDeviceSynchronize()); \
    } while (0)

#define ST_REQUIRE(cond, code, msg)                  \
    do {                                             \
        if (!(cond)) throw ::st::Error((code), (msg)); \
    } while (0)

// runs f at the extern "C" boundary: st::Error -> its code + st_last_error()
template <typename F>
inline int guard(F &&f) {
    try {
        f();
        return ST_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("host allocation failed");
        return ST_ERR_NOMEM;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return ST_ERR_INTERNAL;
    }
}

// ---------------------------------------------------------------------------
// grow-only device workspace, one buffer per named slot
struct Workspace {
    struct Buf {
        void *ptr = nullptr;
        size_t bytes = 0;
    };
    std::map<std::string, Buf> bufs;
    void *get(const std::string &slot, size_t bytes);
    void release();
};

struct StageTimer {
    hipEvent_t ev;
    std::string name;
};

}  // namespace st

struct st_ctx {
    int device = 0;
    // max |x| over the k-means point set, found by check_finite in the same pass as the
    // finiteness test (negative: not known, nd_prepare computes it)
    float km_absmax = -1.0f;
    // the next kmeans_dev's points are finite by construction (the SOG writer's codebook over
    // the SH centroids: data rows and means of finite rows): no finiteness pass and read-back
    bool km_finite_known = false;
    // the N-D k-means point set prepared by nd_prepare (fp16 scale and shape)
    float kn_sigma = 1.0f;
    uint64_t kn_n = 0;
    int kn_d = 0;
    // the last st_dev_kmeans_partials call (member lists kept for st_dev_kmeans_seqsum)
    int ds_nseg = 0, ds_k = 0, ds_d = 0;
    uint64_t ds_n = 0;
    // 1-D partials taken without the member sort (dist_assign_partials1d): the (segment,
    // label) order is built from these only if a pending chain needs it
    const float *ds_pts = nullptr;
    const uint32_t *ds_labels = nullptr;
    bool ds_sorted = true;
    // 1-D k-means: read the uncertified-cluster count back every iteration (set for a rerun
    // after ERR_K1_MANY)
    bool k1_sync = false;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // a second stream of this context (side_stream): independent work of one call that
    // overlaps latency-bound chains on `stream`, joined by the two events
    hipStream_t side = nullptr;
    hipEvent_t side_ev[2] = {nullptr, nullptr};
    // the N-D assign's read-backs: behind the sweep, behind the fix-up (created on first use)
    hipEvent_t kn_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    st::Workspace ws;
    // pinned host staging for small readbacks
    void *pinned = nullptr;
    size_t pinned_bytes = 0;
    // named pinned host buffers (pinned_slot): readbacks queued ahead of the sync that waits for them
    std::map<std::string, std::pair<void *, size_t>> pinned_slots;
    // pinned host buffer of the last .sog archive (st_dev_sog_bundle*)
    void *archive = nullptr;
    size_t archive_bytes = 0;
    // pinned host chunks of the PLY reader
    void *io = nullptr;
    size_t io_bytes = 0;
    // staged host <-> device copies of pageable buffers (staged_h2d / staged_d2h): pinned
    // slots, their events and the host threads that fill / drain them
    void *xfer = nullptr;
    hipEvent_t xfer_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    void *xfer_pool = nullptr;
    std::vector<st::StageTimer> marks;
    bool timing = false;
    std::string last_timings = "{}";
    // the N-D assign's classification summed over the last N-D kmeans_dev call's iterations
    // (st_ctx_last_kmeans_stats): points the sweep decided, pair points, ambiguous points, those
    // whose first candidate list overflowed, those the second list did not hold either (the
    // KdTree walk), and the exact ties walked
    struct KnStats {
        uint64_t assigns = 0, points = 0, pairs = 0, ambiguous = 0, overflow = 0, walked_overflow = 0, ties = 0;
    } kn_stats;
    std::string last_kn_stats = "{}";
    // kernel profiling (st_ctx_set_profiling)
    bool profiling = false;
    struct KEv {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<KEv> kevents;
    std::vector<hipEvent_t> event_pool;
    // side context on the same device (multi-GPU writeSog: rank 0's Morton order runs there)
    st_ctx *aux = nullptr;
    // called by the SOG step once the five textures that precede the SH k-means are queued on
    // the stream (sog_file_dev streams them to the file meanwhile); empty otherwise
    std::function<void(st_ctx *)> sog_early;
    // st_ctx_set_verify: snapshot of the last N-D k-means (prev / final centroids, labels)
    bool verify = false;
    int vf_d = 0, vf_k = 0;
    uint64_t vf_n = 0;
    // host columns whose values are also resident in HBM (workspace slots "plyh.e<element>.c<p>"):
    //  * st_ply_read filled `host` and a host twin `shadow` (every byte as the device copy has it):
    //    the writeSog host forms run on `dev` while other threads compare `host` with `shadow`
    //    (exact: memcmp); a changed byte sends the call back to an upload (st_host_api.hip).  The
    //    twins share one buffer: dropped by the next st_ply_read.  ST_HOST_MIRROR=0: off.
    //  * st_ply_read_resident left `host` unfilled (`lazy`): the values exist only in `dev`, a device
    //    block of the mirror's own (`dev_bytes`), until st_ply_materialize copies them down (the
    //    mirror is then dropped: the caller may change them).  The writeSog host forms read `dev`
    //    directly; every other host form materializes first (the staged copies' bookkeeping).
    //    st_ply_forget drops one whose host memory goes away.  A dropped mirror's block goes to
    //    dev_pool for the next resident read's columns of the same size (freed with the context).
    // mirror_mu guards the list and the pool (the Node addon's finalizers call st_ply_forget from
    // any thread).
    struct HostMirror {
        const void *host;
        uint64_t bytes;
        const void *shadow;  // null when lazy
        const void *dev;
        int element;
        bool lazy;
        uint64_t dev_bytes;  // > 0: dev is this mirror's own block (lazy), returned to dev_pool when dropped
    };
    std::vector<HostMirror> mirrors;
    std::vector<std::pair<void *, uint64_t>> dev_pool;
    std::mutex mirror_mu;
    void *shadow = nullptr;  // the mirrors' host twins (pageable, huge pages, grow-only)
    size_t shadow_bytes = 0;
    // set while a host form runs on mirrors: the compare raises *spec_abort on a mismatch (the
    // N-D k-means checks it every iteration), spec_verdict waits for the compare (true = equal)
    std::atomic<bool> *spec_abort = nullptr;
    std::function<bool()> spec_verdict;
    uint64_t last_reuse_cols = 0, last_reuse_bytes = 0;  // st_ctx_last_host_reuse
    // set by the one-device N-D k-means loop: an assign's pair / ambiguous fix-ups run on the side
    // stream beside the decided points' fix-up (nd_assign_core); ST_FIX_SERIAL=1: one stream
    bool fix_overlap = false;
};

namespace st {

inline void *ws(st_ctx *c, const std::string &slot, size_t bytes) { return c->ws.get(slot, bytes); }
template <typename T>
inline T *wsT(st_ctx *c, const std::string &slot, size_t count) {
    return static_cast<T *>(c->ws.get(slot, count * sizeof(T) + 16));
}
void *pinned(st_ctx *c, size_t bytes);  // host pinned scratch (reused)
hipStream_t side_stream(st_ctx *c);     // c->side, created on first use (non-blocking)
void *pinned_slot(st_ctx *c, const std::string &name, size_t bytes);  // named, grow-only
void *archive_buf(st_ctx *c, size_t bytes);  // host pinned archive buffer (reused, grow-only)
void *io_buf(st_ctx *c, size_t bytes);       // host pinned file-chunk buffer (reused, grow-only)
// copies between pageable host buffers and HBM for the one-call host forms: the bytes move
// through pinned slots that several host threads fill (drain) while the DMA engine moves the
// previous slot, instead of the runtime's single-threaded pageable staging.  Stream-ordered on
// c->stream; both return when every byte has arrived (the host buffers may be reused).
struct HostXfer {
    void *host;
    void *dev;
    size_t bytes;
};
void staged_h2d(st_ctx *c, const std::vector<HostXfer> &xs);
void staged_d2h(st_ctx *c, const std::vector<HostXfer> &xs);
void staged_h2d_raw(st_ctx *c, const std::vector<HostXfer> &xs);  // without the mirrors' bookkeeping
void staged_d2h_raw(st_ctx *c, const std::vector<HostXfer> &xs);  // without the mirrors' bookkeeping
// st_ctx::HostMirror bookkeeping of the staged copies (st_ply.hip): lazy sources are copied down
// before an upload reads them; overwritten destinations stop being mirrors
void mirrors_before_h2d(st_ctx *c, const std::vector<HostXfer> &xs);
void mirrors_before_d2h(st_ctx *c, const std::vector<HostXfer> &xs);
// host-side copy over the context's copy threads (large copies split; small ones inline)
void host_copy(st_ctx *c, char *dst, const char *src, size_t bytes);
// fn(t, nt) on each of the context's nt copy threads; returns when all are done
void host_parallel(st_ctx *c, const std::function<void(int, int)> &fn);
// a speculative host form's gate before it writes anything outside the device: throws SpecAbort
// when the compare found the host columns changed (waits for the compare)
inline void spec_gate(st_ctx *c) {
    if (c->spec_verdict && !c->spec_verdict()) throw SpecAbort();
}
void use_device(st_ctx *c);
void mark(st_ctx *c, const char *name);  // records a hipEvent when timing is on

// brackets one kernel launch with hipEvents when profiling is enabled
struct KTimer {
    st_ctx *c;
    hipEvent_t a = nullptr, b = nullptr;
    const char *name;
    hipStream_t s;  // the stream the timed kernels run on (the context's unless given)
    KTimer(st_ctx *ctx, const char *nm, hipStream_t stream = nullptr);
    ~KTimer();
};

inline unsigned grid_for(uint64_t work, unsigned per_block, unsigned cap = 1u << 30) {
    uint64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---------------------------------------------------------------------------
// primitives (st_prims.hip)

// exclusive scan of n u32 values (out may alias in); returns nothing, total written to *d_total if not null
void scan_u32(st_ctx *c, const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *d_total);

// stable LSD radix sort of (key, value) pairs on bits [begin_bit, end_bit)
void radix_sort_u32(st_ctx *c, uint32_t *keys, uint32_t *vals, uint64_t n, int begin_bit, int end_bit,
                    const std::string &tag);
// the same from read-only keys with the identity permutation as values, into out_keys / out_vals
void radix_sort_u32_iota(st_ctx *c, const uint32_t *in_keys, uint64_t n, int begin_bit, int end_bit,
                         uint32_t *out_keys, uint32_t *out_vals, const std::string &tag);
// the general form: in_vals null = the identity permutation; out_vals may alias in_vals when the
// pass count is even (the first pass writes the scratch pair).  hist0, when not null, holds the
// first digit's per-tile counts in the sort's layout (count of digit d in tile t at
// d * radix_tiles(n) + t, tiles of RADIX_TILE elements), produced by the caller's key kernel;
// it is scanned in place and reused as the histogram buffer of the later passes
constexpr int RADIX_TILE = 4096;
inline uint32_t radix_tiles(uint64_t n) { return (uint32_t)((n + RADIX_TILE - 1) / RADIX_TILE); }
void radix_sort_u32_from(st_ctx *c, const uint32_t *in_keys, const uint32_t *in_vals, uint64_t n, int begin_bit,
                         int end_bit, uint32_t *out_keys, uint32_t *out_vals, uint32_t *hist0, const std::string &tag);
// as radix_sort_u32, but the result stays in whichever buffer pair the last pass wrote
// (the caller's or the workspace's): *out_keys / *out_vals point at it
void radix_sort_u32_inplace_or_swap(st_ctx *c, uint32_t *keys, uint32_t *vals, uint64_t n, int b0, int b1,
                                    const std::string &tag, uint32_t **out_keys, uint32_t **out_vals);
void radix_sort_u64(st_ctx *c, uint64_t *keys, uint32_t *vals, uint64_t n, int begin_bit, int end_bit,
                    const std::string &tag);

// iota
// min and max of each column as order-preserving u32 keys (NaN ignored; an all-NaN or empty
// column gives min 0xffffffff, max 0): out[2a] = min, out[2a + 1] = max.  cols: host array of
// device pointers, ncols <= 64
void minmax_keys_dev(st_ctx *c, const float *const *cols, int ncols, uint64_t n, uint32_t *out);
void iota_u32(st_ctx *c, uint32_t *out, uint64_t n);

// column lookups on an st_table
int find_col(const st_table *t, const char *name);
float *col_or_null(const st_table *t, const char *name);
int sh_coeffs_of(const st_table *t);  // band rule: transform.ts:20 / write-sog.ts:296

// module entry points (device pointers)
void transform_dev(st_ctx *c, const st_table *t, const st_transform_params *p);
uint64_t filter_finite_dev(st_ctx *c, const st_table *t, uint32_t *out_idx);
void permute_rows_dev(st_ctx *c, const st_table *src, const uint32_t *idx, uint64_t m, const st_table *dst);
void concat_rows_dev(st_ctx *c, const st_table *const *srcs, int nsrc, const st_table *dst);
// typed tables (st_table.hip)
int type_size(int32_t st_ply_type);  // 0 for an unknown code
uint64_t filter_finite_tdev(st_ctx *c, const st_ttable *t, uint32_t *out_idx);
// stable compaction: out_idx = the rows with flags[i] != 0, ascending; returns their count (syncs)
uint64_t compact_flags_dev(st_ctx *c, const uint32_t *flags, uint64_t n, uint32_t *out_idx);
uint64_t filter_value_tdev(st_ctx *c, const st_ttable *t, const char *column, int32_t cmp, double value,
                           uint32_t *out_idx);
void permute_rows_tdev(st_ctx *c, const st_ttable *src, const uint32_t *idx, uint64_t m, const st_ttable *dst);
int combine_layout(const st_ttable *const *srcs, int nsrc, int32_t *col_table, int32_t *col_index);
void combine_tdev(st_ctx *c, const st_ttable *const *srcs, int nsrc, const st_ttable *dst);
void morton_order_dev(st_ctx *c, const float *x, const float *y, const float *z, uint32_t *indices, uint64_t n);
void morton_order_dev_f64(st_ctx *c, const double *x, const double *y, const double *z, uint32_t *indices,
                          uint64_t n);
// x / y / z of any column types (ST_PLY_*): float64 keys when any is not float32 (st_morton.hip)
void morton_order_tdev(st_ctx *c, const void *const xyz[3], const int32_t types[3], uint32_t *indices, uint64_t n);
// transform() over a typed table in place (st_transform.hip)
void transform_tdev(st_ctx *c, const st_ttable *t, const st_transform_params *p);
// (sh64: the 3 sh_coeffs SH columns' JS numbers as float64 when they are not all float32; the
// SH bytes are computed from those and t's f_rest columns are not read)
void pack_compressed_dev(st_ctx *c, const st_table *t, const uint32_t *order, float *chunk, uint32_t *vertex,
                         uint8_t *sh, const double *const *sh64 = nullptr, int sh_coeffs = 0);
// returns draws consumed
// initializeCentroids over a table of n rows: rows (device) = the k distinct floor(draw * n) in
// draw order, *used = draws consumed (device window with the host loop as fallback)
void kmeans_init_rows(st_ctx *c, const double *draws, uint64_t ndraws, uint64_t n, int k, uint32_t *rows,
                      uint64_t *used);
// out[c * k + i] = cols[c][rows[i] - offset] where offset <= rows[i] < offset + n_local, bits 0 elsewhere
void gather_owned_rows(st_ctx *c, const float *const *cols, int d, uint64_t n_local, uint64_t offset,
                       const uint32_t *rows, int k, float *out);
// (host_init: initializeCentroids by the host's loop instead of on the device)
// (sum64: float64 columns (host array of device pointers) summed by calcAverage instead of cols:
// the JS numbers of columns that are not float32, D > 1)
uint64_t kmeans_dev(st_ctx *c, const float *const *cols, int d, uint64_t n, int k, int iters, const double *draws,
                    uint64_t ndraws, float *centroids, uint32_t *labels, bool host_init = false,
                    const double *const *sum64 = nullptr);
// st_ctx_last_kmeans_stats' JSON from c->kn_stats (the N-D k-means writers call it at their end)
void kn_stats_publish(st_ctx *c);
uint64_t cluster1d_dev(st_ctx *c, const float *const *cols, int ncols, uint64_t n, int iters, const double *draws,
                       uint64_t ndraws, float *centroids256, uint8_t *labels);
uint64_t sog_dev(st_ctx *c, const st_table *t, int iters, const double *draws, uint64_t ndraws, st_sog_meta *meta,
                 const st_sog_textures *out);
// writeSog's device part over a table of any column types (write-sog.ts reads the members as JS
// numbers, cluster1d and the k-means points through Float32Arrays): float32 tables take sog_dev
uint64_t sog_tdev(st_ctx *c, const st_ttable *t, int iters, const double *draws, uint64_t ndraws,
                  st_sog_meta *meta, const st_sog_textures *out);
void codebook_dev(st_ctx *c, const float *cen, const uint32_t *lab, uint64_t total, float *centroids256,
                  uint8_t *labels);
void sog_scatter_dev(st_ctx *c, const st_table *t, const uint32_t *pos, const double lo[3], const double hi[3],
                     const uint8_t *scale_lab, const uint8_t *color_lab, const uint32_t *shn_lab, st_sog_meta *meta,
                     const st_sog_textures *out);
void shn_centroids_dev(st_ctx *c, const uint8_t *cl, int C, int pal, uint8_t *out);
// the scales / sh0 texels of n rows in row order (byte labels: three planes of n; opacity nullable)
void sog_table_rows(st_ctx *c, uint64_t n, const uint8_t *lab, const float *opacity, uint8_t *out);
// cluster1d of the scales (a) and the colours (b) as the single-device writer runs them (b beside a
// on the context `side`, speculatively from draw 0); returns the draws both took
uint64_t cluster1d_pair_dev(st_ctx *c, st_ctx *side, const float *const *a, const float *const *b, uint64_t n,
                            int iters, const double *draws, uint64_t ndraws, float *cb_a, uint8_t *lab_a, float *cb_b,
                            uint8_t *lab_b);

// PLY ingest / compressed-PLY reader (st_ply.hip)
// a host consumer of the PLY reader's pinned row chunks (st_ply_read's host transpose)
struct ChunkSink {
    virtual ~ChunkSink() = default;
    // rows [row, row + nrows) of the element are in the pinned chunk buffer b (0 / 1): consume
    // them asynchronously
    virtual void take(int b, const uint8_t *rows, uint64_t row, uint64_t nrows) = 0;
    // before buffer b is refilled: returns once the host is done with its last chunk
    virtual void wait(int b) = 0;
};
void ply_read_dev(st_ctx *c, int fd, const st_ply_header &h, int element, void *const *cols,
                  ChunkSink *sink = nullptr);
// st_ply_read: into the caller's host columns, and the element's mirrors (st_ctx::HostMirror)
void ply_read_host(st_ctx *c, int fd, const st_ply_header &h, int element, void *const *host_cols, bool lazy = false);
// st_ply_materialize: the lazy mirrors among these host columns copied down and dropped (upload()
// calls it first: no host form reads an unfilled column)
void materialize_lazy(st_ctx *c, const void *const *host, int n);
// (mirror_mu held) the mirrors `pick` selects removed, their own device blocks pooled
void drop_mirrors_locked(st_ctx *c, const std::function<bool(const st_ctx::HostMirror &)> &pick);
void decompress_ply_dev(st_ctx *c, uint64_t n, const float *const *chunk, const uint32_t *const *vertex,
                        const uint8_t *const *sh, int nsh, float *const *out);

// multi-GPU building blocks (st_dist.hip)
void minmax_dev(st_ctx *c, const float *const *cols, int ncols, uint64_t n, double *lo, double *hi);
void dist_prepare(st_ctx *c, const float *const *cols, int d, uint64_t n);
void dist_assign(st_ctx *c, const float *const *cols, int d, uint64_t n, int k, const float *cen, uint32_t *labels);
// dist_assign + dist_partials of a 1-D point set with k <= 256 in one pass (no member sort)
void dist_assign_partials1d(st_ctx *c, const float *pts, uint64_t n, int nseg, int k, const float *cen,
                            uint32_t *labels, double *sums, double *sabs, int32_t *emin, uint32_t *counts);
// dist_assign + dist_partials of an N-D shard (one segment) in one pass: the fused fix-up's
// sums, the member order built only for pending pairs; false (nothing written but the labels):
// the assign could not fuse, the caller takes dist_partials
// (dcols: the shard's column pointers, a device array)
bool dist_assign_partials_nd(st_ctx *c, const float *const *dcols, int d, uint64_t n, int k, const float *cen,
                             uint32_t *labels, double *sums, double *sabs, int32_t *emin, uint32_t *counts);
void dist_partials(st_ctx *c, const float *const *cols, int d, uint64_t n, int nseg, int k, const uint32_t *labels,
                   double *sums, double *sabs, int32_t *emin, uint32_t *counts);
void dist_seqsum(st_ctx *c, int d, int k, int seg, const uint32_t *pairs, uint32_t npairs, double *running,
                 const int32_t *emin, const double *sabs);
uint32_t dist_finish(st_ctx *c, int d, int k, const double *sums, const double *sabs, const int32_t *emin,
                     const uint32_t *counts, float *cen, uint32_t *pending);
void dist_average(st_ctx *c, int d, int k, const uint32_t *pairs, uint32_t npairs, const double *running,
                  const uint32_t *counts, float *cen);

// processDataTable on a device float32 table (st_chain.hip)
struct ProcessedF32 {
    std::vector<std::string> names;
    std::vector<const char *> cn;
    std::vector<float *> cols;
    st_table t{};
};
void chain_apply_f32(st_ctx *c, const st_table *in, const st_action *actions, int nactions, const std::string &tag,
                     ProcessedF32 &out);

// multi-GPU writeSog (st_multi.hip): the st_set_devices group (empty: one device); the returned
// reference keeps the group alive for the caller's call even if st_set_devices replaces it
std::shared_ptr<st_group> default_group();
int apply_env_devices();  // ST_NUM_GPUS on first use; ST_OK or the error (st_last_error set)

}  // namespace st
