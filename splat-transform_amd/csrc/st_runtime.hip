// st_runtime.hip -- context, workspace, error plumbing, table helpers.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <sstream>
#include <thread>

#include "st_internal.h"
#include "st_webp.h"

namespace st {

static thread_local std::string g_last_error;
bool g_sync_check = false;

void set_last_error(const std::string &msg) { g_last_error = msg; }

void *Workspace::get(const std::string &slot, size_t bytes) {
    if (bytes == 0) bytes = 16;
    Buf &b = bufs[slot];
    if (b.bytes < bytes) {
        if (b.ptr) ST_HIP(hipFree(b.ptr));
        b.ptr = nullptr;
        b.bytes = 0;
        size_t want = bytes + bytes / 8;  // headroom for slowly growing sizes
        hipError_t e = hipMalloc(&b.ptr, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            throw Error(ST_ERR_NOMEM, "workspace '" + slot + "': hipMalloc(" + std::to_string(want) + ") failed");
        }
        b.bytes = want;
    }
    return b.ptr;
}

void Workspace::release() {
    for (auto &kv : bufs)
        if (kv.second.ptr) (void)hipFree(kv.second.ptr);
    bufs.clear();
}

void *pinned(st_ctx *c, size_t bytes) {
    if (c->pinned_bytes < bytes) {
        if (c->pinned) ST_HIP(hipHostFree(c->pinned));
        c->pinned = nullptr;
        ST_HIP(hipHostMalloc(&c->pinned, bytes, hipHostMallocDefault));
        c->pinned_bytes = bytes;
    }
    return c->pinned;
}

hipStream_t side_stream(st_ctx *c) {
    if (!c->side) {
        ST_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        for (auto &e : c->side_ev) ST_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    return c->side;
}

void *pinned_slot(st_ctx *c, const std::string &name, size_t bytes) {
    auto &b = c->pinned_slots[name];
    if (b.second < bytes) {
        if (b.first) ST_HIP(hipHostFree(b.first));
        b.first = nullptr;
        b.second = 0;
        ST_HIP(hipHostMalloc(&b.first, bytes, hipHostMallocDefault));
        b.second = bytes;
    }
    return b.first;
}

void *archive_buf(st_ctx *c, size_t bytes) {
    if (c->archive_bytes < bytes) {
        if (c->archive) ST_HIP(hipHostFree(c->archive));
        c->archive = nullptr;
        c->archive_bytes = 0;
        const size_t want = bytes + bytes / 8;
        ST_HIP(hipHostMalloc(&c->archive, want, hipHostMallocDefault));
        c->archive_bytes = want;
    }
    return c->archive;
}

void *io_buf(st_ctx *c, size_t bytes) {
    if (c->io_bytes < bytes) {
        if (c->io) ST_HIP(hipHostFree(c->io));
        c->io = nullptr;
        c->io_bytes = 0;
        ST_HIP(hipHostMalloc(&c->io, bytes, hipHostMallocDefault));
        c->io_bytes = bytes;
    }
    return c->io;
}

void use_device(st_ctx *c) { ST_HIP(hipSetDevice(c->device)); }

// ---- staged pageable copies ----------------------------------------------------------
namespace {
constexpr int XF_SLOTS = 4;                 // pinned slots (st_ctx::xfer_ev)
// bytes per slot and host threads copying one slot (ST_XFER_CHUNK_MB / ST_XFER_THREADS: experiments)
// (clamped when parsed: a zero chunk would make the piece loop below spin forever)
const size_t XF_CHUNK = std::max<size_t>(1, std::min<size_t>(1024, getenv("ST_XFER_CHUNK_MB") ?
    std::strtoull(getenv("ST_XFER_CHUNK_MB"), nullptr, 10) : 16ull)) << 20;
const int XF_THREADS = std::max(1, std::min(64, getenv("ST_XFER_THREADS") ? std::atoi(getenv("ST_XFER_THREADS")) : 8));
constexpr size_t XF_DIRECT = 1ull << 20;     // smaller copies go through the runtime as they are

// host threads that run one job at a time, each thread taking its share
struct CopyPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go, done;
    std::function<void(int)> job;
    uint64_t gen = 0;
    int left = 0;
    bool stop = false;
    explicit CopyPool(int n) {
        for (int i = 0; i < n; ++i)
            th.emplace_back([this, i] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(int)> j;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        go.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        j = job;
                    }
                    j(i);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--left == 0) done.notify_all();
                }
            });
    }
    void run(std::function<void(int)> f) {
        std::unique_lock<std::mutex> lk(mu);
        job = std::move(f);
        left = (int)th.size();
        ++gen;
        go.notify_all();
        done.wait(lk, [&] { return left == 0; });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        go.notify_all();
        for (auto &t : th) t.join();
    }
};

struct Piece {
    char *host, *dev;
    size_t bytes;
};

void xfer_setup(st_ctx *c) {
    ST_REQUIRE(XF_CHUNK > 0 && XF_THREADS > 0, ST_ERR_ARG, "ST_XFER_CHUNK_MB / ST_XFER_THREADS must be positive");
    if (!c->xfer) ST_HIP(hipHostMalloc(&c->xfer, XF_SLOTS * XF_CHUNK, hipHostMallocDefault));
    for (auto &e : c->xfer_ev)
        if (!e) ST_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c->xfer_pool) c->xfer_pool = new CopyPool(XF_THREADS);
}


// the staged transfers cut into slot-sized pieces; small ones are issued directly
std::vector<Piece> pieces_of(st_ctx *c, const std::vector<HostXfer> &xs, bool h2d) {
    std::vector<Piece> ps;
    for (const auto &x : xs) {
        if (!x.bytes) continue;
        if (x.bytes < XF_DIRECT) {
            if (h2d) ST_HIP(hipMemcpyAsync(x.dev, x.host, x.bytes, hipMemcpyHostToDevice, c->stream));
            else ST_HIP(hipMemcpyAsync(x.host, x.dev, x.bytes, hipMemcpyDeviceToHost, c->stream));
            continue;
        }
        for (size_t o = 0; o < x.bytes; o += XF_CHUNK)
            ps.push_back(Piece{static_cast<char *>(x.host) + o, static_cast<char *>(x.dev) + o,
                               std::min(XF_CHUNK, x.bytes - o)});
    }
    return ps;
}
}  // namespace

// host-side copy of one piece: split over the pool when it is large
void host_copy(st_ctx *c, char *dst, const char *src, size_t bytes) {
    if (bytes < (2ull << 20)) {
        std::memcpy(dst, src, bytes);
        return;
    }
    if (!c->xfer_pool) c->xfer_pool = new CopyPool(XF_THREADS);
    static_cast<CopyPool *>(c->xfer_pool)->run([=](int t) {
        const size_t a0 = bytes * t / XF_THREADS, a1 = bytes * (t + 1) / XF_THREADS;
        std::memcpy(dst + a0, src + a0, a1 - a0);
    });
}

void host_parallel(st_ctx *c, const std::function<void(int, int)> &fn) {
    if (!c->xfer_pool) c->xfer_pool = new CopyPool(XF_THREADS);
    static_cast<CopyPool *>(c->xfer_pool)->run([&fn](int t) { fn(t, XF_THREADS); });
}

// ST_XFER_PRINT=1: bytes and rate of every staged copy on stderr
struct XferLog {
    const char *what;
    const std::vector<HostXfer> &xs;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~XferLog() {
        if (!getenv("ST_XFER_PRINT")) return;
        size_t b = 0;
        for (auto &x : xs) b += x.bytes;
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        fprintf(stderr, "[st xfer] %s %.1f MB in %.2f ms = %.1f GB/s\n", what, b / 1e6, s * 1e3, b / s / 1e9);
    }
};

void staged_h2d(st_ctx *c, const std::vector<HostXfer> &xs) {
    mirrors_before_h2d(c, xs);
    staged_h2d_raw(c, xs);
}

void staged_h2d_raw(st_ctx *c, const std::vector<HostXfer> &xs) {
    XferLog log{"h2d", xs};
    std::vector<Piece> ps = pieces_of(c, xs, true);
    if (!ps.empty()) {
        xfer_setup(c);
        bool pending[XF_SLOTS] = {false, false, false, false};
        for (size_t k = 0; k < ps.size(); ++k) {
            const int b = (int)(k % XF_SLOTS);
            char *slot = static_cast<char *>(c->xfer) + b * XF_CHUNK;
            if (pending[b]) ST_HIP(hipEventSynchronize(c->xfer_ev[b]));  // the slot's last DMA is done
            host_copy(c, slot, ps[k].host, ps[k].bytes);
            ST_HIP(hipMemcpyAsync(ps[k].dev, slot, ps[k].bytes, hipMemcpyHostToDevice, c->stream));
            ST_HIP(hipEventRecord(c->xfer_ev[b], c->stream));
            pending[b] = true;
        }
    }
    ST_HIP(hipStreamSynchronize(c->stream));
}

void staged_d2h(st_ctx *c, const std::vector<HostXfer> &xs) {
    mirrors_before_d2h(c, xs);
    staged_d2h_raw(c, xs);
}

void staged_d2h_raw(st_ctx *c, const std::vector<HostXfer> &xs) {
    XferLog log{"d2h", xs};
    std::vector<Piece> ps = pieces_of(c, xs, false);
    if (!ps.empty()) {
        xfer_setup(c);
        long held[XF_SLOTS] = {-1, -1, -1, -1};  // the piece whose bytes wait in each slot
        auto drain = [&](int b) {
            if (held[b] < 0) return;
            ST_HIP(hipEventSynchronize(c->xfer_ev[b]));
            const Piece &p = ps[(size_t)held[b]];
            host_copy(c, p.host, static_cast<char *>(c->xfer) + b * XF_CHUNK, p.bytes);
            held[b] = -1;
        };
        for (size_t k = 0; k < ps.size(); ++k) {
            const int b = (int)(k % XF_SLOTS);
            drain(b);
            ST_HIP(hipMemcpyAsync(static_cast<char *>(c->xfer) + b * XF_CHUNK, ps[k].dev, ps[k].bytes,
                                  hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipEventRecord(c->xfer_ev[b], c->stream));
            held[b] = (long)k;
        }
        for (size_t k = ps.size() > XF_SLOTS ? ps.size() - XF_SLOTS : 0; k < ps.size(); ++k) drain((int)(k % XF_SLOTS));
    }
    ST_HIP(hipStreamSynchronize(c->stream));
}

void mark(st_ctx *c, const char *name) {
    if (!c->timing) return;
    StageTimer t;
    t.name = name;
    ST_HIP(hipEventCreate(&t.ev));
    ST_HIP(hipEventRecord(t.ev, c->stream));
    c->marks.push_back(t);
}

static hipEvent_t pool_event(st_ctx *c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    ST_HIP(hipEventCreate(&e));
    return e;
}

KTimer::KTimer(st_ctx *ctx, const char *nm, hipStream_t stream) : c(ctx), name(nm), s(stream ? stream : ctx->stream) {
    if (!c->profiling) return;
    a = pool_event(c);
    b = pool_event(c);
    ST_HIP(hipEventRecord(a, s));
}

KTimer::~KTimer() {
    if (!a) return;
    if (hipEventRecord(b, s) == hipSuccess) c->kevents.push_back({name, a, b});
}

static void begin_timing(st_ctx *c) {
    c->timing = getenv("ST_TIMING") != nullptr;
    for (auto &m : c->marks) (void)hipEventDestroy(m.ev);
    c->marks.clear();
    mark(c, "begin");
}

static void end_timing(st_ctx *c) {
    if (!c->timing) return;
    mark(c, "end");
    ST_HIP(hipEventSynchronize(c->marks.back().ev));
    // per name: the sum of its intervals (the time since the previous mark, over every time the
    // stage ran: a k-means iteration marks each pass); "sog.*" names mark writeSog's top-level
    // stages and take the interval since the previous "sog.*" mark, nested marks included
    std::vector<std::string> order;
    std::map<std::string, double> tot;
    size_t top = 0;
    for (size_t i = 1; i < c->marks.size(); ++i) {
        const std::string &nm = c->marks[i].name;
        const bool is_top = nm.compare(0, 4, "sog.") == 0;
        float ms = 0;
        ST_HIP(hipEventElapsedTime(&ms, c->marks[is_top ? top : i - 1].ev, c->marks[i].ev));
        if (!tot.count(nm)) order.push_back(nm);
        tot[nm] += ms;
        if (is_top) top = i;
    }
    std::ostringstream os;
    os << "{";
    for (size_t i = 0; i < order.size(); ++i) os << (i ? ", " : "") << "\"" << order[i] << "\": " << tot[order[i]];
    os << "}";
    c->last_timings = os.str();
    if (getenv("ST_TIMING_PRINT")) fprintf(stderr, "[st timing] %s\n", c->last_timings.c_str());
}

int find_col(const st_table *t, const char *name) {
    for (int i = 0; i < t->ncol; ++i)
        if (t->names[i] && strcmp(t->names[i], name) == 0) return i;
    return -1;
}

float *col_or_null(const st_table *t, const char *name) {
    int i = find_col(t, name);
    return i < 0 ? nullptr : t->cols[i];
}

int sh_coeffs_of(const st_table *t) {
    // { '9': 1, '24': 2, '-1': 3 }[index of first missing f_rest_i] ?? 0
    int first_missing = -1;
    char nm[32];
    for (int i = 0; i < 45; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        if (find_col(t, nm) < 0) {
            first_missing = i;
            break;
        }
    }
    switch (first_missing) {
        case 9: return 3;
        case 24: return 8;
        case -1: return 15;
        default: return 0;
    }
}

}  // namespace st

// ---------------------------------------------------------------------------
// extern "C" boundary
using namespace st;

template <typename F>
static int guarded(F &&f) {
    try {
        f();
        return ST_OK;
    } catch (const st::Error &e) {
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

#define ST_ARG(cond, msg) ST_REQUIRE(cond, ST_ERR_ARG, msg)

static void check_table(const st_table *t) {
    ST_ARG(t != nullptr, "table is NULL");
    ST_ARG(t->ncol >= 0 && (t->ncol == 0 || (t->names && t->cols)), "table: bad column arrays");
    for (int i = 0; i < t->ncol; ++i) ST_ARG(t->cols[i] != nullptr || t->n == 0, "table: NULL column pointer");
}

extern "C" {

int st_abi_version(void) { return ST_ABI_VERSION; }

const char *st_last_error(void) { return g_last_error.c_str(); }

int st_device_count(int32_t *count) {
    return guarded([&] {
        ST_ARG(count, "count is NULL");
        int n = 0;
        ST_HIP(hipGetDeviceCount(&n));
        *count = n;
    });
}

int st_ctx_create(int32_t device, st_ctx **out) {
    return guarded([&] {
        ST_ARG(out, "out is NULL");
        int n = 0;
        ST_HIP(hipGetDeviceCount(&n));
        ST_REQUIRE(n > 0, ST_ERR_HIP, "no HIP device visible (the MI355X product path has no CPU fallback)");
        g_sync_check = getenv("ST_SYNC_CHECK") != nullptr;
        ST_ARG(device >= 0 && device < n, "device index out of range");
        hipDeviceProp_t prop;
        ST_HIP(hipGetDeviceProperties(&prop, device));
        ST_REQUIRE(strncmp(prop.gcnArchName, "gfx950", 6) == 0, ST_ERR_UNSUPPORTED,
                   std::string("libsplat_hip is built for gfx950 (MI355X); device is ") + prop.gcnArchName);
        auto *c = new st_ctx();
        c->device = device;
        ST_HIP(hipSetDevice(device));
        ST_HIP(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
        c->stream = c->own_stream;
        *out = c;
    });
}

void st_ctx_destroy(st_ctx *c) {
    if (!c) return;
    st_ctx_destroy(c->aux);
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->ws.release();
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->archive) (void)hipHostFree(c->archive);
    if (c->io) (void)hipHostFree(c->io);
    std::free(c->shadow);
    for (auto &m : c->mirrors)
        if (m.dev_bytes) (void)hipFree(const_cast<void *>(m.dev));
    for (auto &b : c->dev_pool) (void)hipFree(b.first);
    if (c->xfer) (void)hipHostFree(c->xfer);
    for (auto &kv : c->pinned_slots)
        if (kv.second.first) (void)hipHostFree(kv.second.first);
    for (auto e : c->xfer_ev)
        if (e) (void)hipEventDestroy(e);
    delete static_cast<CopyPool *>(c->xfer_pool);
    for (auto &m : c->marks) (void)hipEventDestroy(m.ev);
    for (auto &k : c->kevents) {
        (void)hipEventDestroy(k.a);
        (void)hipEventDestroy(k.b);
    }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    if (c->side) {
        (void)hipStreamSynchronize(c->side);
        (void)hipStreamDestroy(c->side);
    }
    for (auto e : c->side_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : c->kn_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int st_ctx_set_stream(st_ctx *c, void *s) {
    return guarded([&] {
        ST_ARG(c, "ctx is NULL");
        use_device(c);
        if (s) {
            // the caller's stream replaces the context's own: release it (one hardware queue fewer;
            // GPU_MAX_HW_QUEUES bounds them per process)
            if (c->own_stream) {
                ST_HIP(hipStreamSynchronize(c->own_stream));
                ST_HIP(hipStreamDestroy(c->own_stream));
                c->own_stream = nullptr;
            }
            c->stream = (hipStream_t)s;
        } else {
            if (!c->own_stream) ST_HIP(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
            c->stream = c->own_stream;
        }
    });
}

int st_ctx_synchronize(st_ctx *c) {
    return guarded([&] {
        ST_ARG(c, "ctx is NULL");
        use_device(c);
        ST_HIP(hipStreamSynchronize(c->stream));
    });
}

const char *st_ctx_last_timings(st_ctx *c) { return c ? c->last_timings.c_str() : "{}"; }
const char *st_ctx_last_kmeans_stats(st_ctx *c) { return c ? c->last_kn_stats.c_str() : "{}"; }

int st_ctx_last_host_reuse(st_ctx *c, uint64_t *columns, uint64_t *bytes) {
    return guarded([&] {
        ST_ARG(c && columns && bytes, "NULL argument");
        *columns = c->last_reuse_cols;
        *bytes = c->last_reuse_bytes;
    });
}

int st_ctx_set_profiling(st_ctx *c, int32_t enable) {
    return guarded([&] {
        ST_ARG(c, "ctx is NULL");
        c->profiling = enable != 0;
    });
}

int st_ctx_reset_kernel_stats(st_ctx *c) {
    return guarded([&] {
        ST_ARG(c, "ctx is NULL");
        use_device(c);
        ST_HIP(hipStreamSynchronize(c->stream));
        for (auto &k : c->kevents) {
            c->event_pool.push_back(k.a);
            c->event_pool.push_back(k.b);
        }
        c->kevents.clear();
    });
}

int st_ctx_kernel_stats(st_ctx *c, const char *name, double *total_ms, uint64_t *launches) {
    return guarded([&] {
        ST_ARG(c && name && total_ms && launches, "NULL argument");
        use_device(c);
        double t = 0;
        uint64_t cnt = 0;
        for (auto &k : c->kevents) {
            if (k.name != name) continue;
            ST_HIP(hipEventSynchronize(k.b));
            float ms = 0;
            ST_HIP(hipEventElapsedTime(&ms, k.a, k.b));
            t += ms;
            ++cnt;
        }
        *total_ms = t;
        *launches = cnt;
    });
}

int st_ctx_set_verify(st_ctx *c, int32_t enable) {
    return guarded([&] {
        ST_ARG(c, "ctx is NULL");
        c->verify = enable != 0;
    });
}

int st_ctx_verify_snapshot(st_ctx *c, float *prev, float *cen, uint32_t *labels, int32_t *d, int32_t *k,
                           uint64_t *n) {
    return guarded([&] {
        ST_ARG(c && d && k && n, "NULL argument");
        ST_REQUIRE(c->vf_k > 0, ST_ERR_ARG, "no k-means snapshot (st_ctx_set_verify before the call)");
        use_device(c);
        const size_t cbytes = (size_t)c->vf_k * c->vf_d * sizeof(float);
        const struct {
            void *dst;
            const char *slot;
            size_t bytes;
        } parts[3] = {{prev, "verify.prev", cbytes}, {cen, "verify.cen", cbytes}, {labels, "verify.labels", c->vf_n * 4}};
        for (auto &p : parts)
            if (p.dst) ST_HIP(hipMemcpyAsync(p.dst, ws(c, p.slot, p.bytes), p.bytes, hipMemcpyDeviceToDevice, c->stream));
        *d = c->vf_d;
        *k = c->vf_k;
        *n = c->vf_n;
    });
}

// ---- device entry points --------------------------------------------------
int st_dev_transform(st_ctx *c, const st_table *t, const st_transform_params *p) {
    return guarded([&] {
        ST_ARG(c && p, "NULL argument");
        check_table(t);
        use_device(c);
        transform_dev(c, t, p);
    });
}

int st_dev_transform_t(st_ctx *c, const st_ttable *t, const st_transform_params *p) {
    return guarded([&] {
        ST_REQUIRE(c && t && p && (t->ncol == 0 || (t->names && t->types && t->cols)), ST_ERR_ARG, "NULL argument");
        use_device(c);
        transform_tdev(c, t, p);
    });
}

int st_dev_morton_order_t(st_ctx *c, const void *const xyz[3], const int32_t types[3], uint32_t *idx, uint64_t n) {
    return guarded([&] {
        ST_REQUIRE(c && xyz && types && ((xyz[0] && xyz[1] && xyz[2] && idx) || n == 0), ST_ERR_ARG, "NULL argument");
        for (int a = 0; a < 3; ++a) ST_REQUIRE(type_size(types[a]) > 0, ST_ERR_ARG, "morton: bad column type");
        use_device(c);
        morton_order_tdev(c, xyz, types, idx, n);
    });
}

int st_dev_filter_finite(st_ctx *c, const st_table *t, uint32_t *out_idx, uint64_t *out_n) {
    return guarded([&] {
        ST_ARG(c && out_n, "NULL argument");
        check_table(t);
        use_device(c);
        *out_n = filter_finite_dev(c, t, out_idx);
    });
}

int st_dev_permute_rows(st_ctx *c, const st_table *src, const uint32_t *idx, uint64_t m, const st_table *dst) {
    return guarded([&] {
        ST_ARG(c && (idx || m == 0), "NULL argument");
        check_table(src);
        check_table(dst);
        ST_ARG(dst->ncol == src->ncol && dst->n == m, "permute_rows: dst must have src's columns and m rows");
        use_device(c);
        permute_rows_dev(c, src, idx, m, dst);
    });
}

int st_dev_concat_rows(st_ctx *c, const st_table *const *srcs, int32_t nsrc, const st_table *dst) {
    return guarded([&] {
        ST_ARG(c && srcs && nsrc > 0, "NULL argument");
        for (int i = 0; i < nsrc; ++i) check_table(srcs[i]);
        check_table(dst);
        use_device(c);
        concat_rows_dev(c, srcs, nsrc, dst);
    });
}

static void check_ttable(const st_ttable *t) {
    ST_ARG(t != nullptr, "table is NULL");
    ST_ARG(t->ncol >= 0 && (t->ncol == 0 || (t->names && t->types && t->cols)), "table: bad column arrays");
    for (int i = 0; i < t->ncol; ++i) {
        ST_ARG(t->names[i] && (t->cols[i] || t->n == 0), "table: NULL column");
        ST_ARG(type_size(t->types[i]) > 0, std::string("table: column ") + t->names[i] + " has an unknown type");
        ST_ARG(((uintptr_t)t->cols[i] % type_size(t->types[i])) == 0,
               std::string("table: column ") + t->names[i] + " is not aligned to its element size");
    }
}

int st_dev_filter_finite_t(st_ctx *c, const st_ttable *t, uint32_t *out_idx, uint64_t *out_n) {
    return guarded([&] {
        ST_ARG(c && out_n && (out_idx || (t && t->n == 0)), "NULL argument");
        check_ttable(t);
        use_device(c);
        *out_n = filter_finite_tdev(c, t, out_idx);
    });
}

int st_dev_permute_rows_t(st_ctx *c, const st_ttable *src, const uint32_t *idx, uint64_t m, const st_ttable *dst) {
    return guarded([&] {
        ST_ARG(c && (idx || m == 0), "NULL argument");
        check_ttable(src);
        check_ttable(dst);
        ST_ARG(dst->ncol == src->ncol && dst->n == m, "permute_rows: dst must have src's columns and m rows");
        for (int i = 0; i < src->ncol; ++i)
            ST_ARG(src->types[i] == dst->types[i], "permute_rows: dst column types differ from src");
        use_device(c);
        permute_rows_tdev(c, src, idx, m, dst);
    });
}

int st_combine_layout(const st_ttable *const *srcs, int32_t nsrc, int32_t *col_table, int32_t *col_index,
                      int32_t *ncol) {
    return guarded([&] {
        ST_ARG(srcs && nsrc > 0 && ncol, "NULL argument");
        for (int i = 0; i < nsrc; ++i) {
            ST_ARG(srcs[i] && srcs[i]->ncol >= 0 && (srcs[i]->ncol == 0 || (srcs[i]->names && srcs[i]->types)),
                   "combine_layout: bad table");
        }
        *ncol = combine_layout(srcs, nsrc, col_table, col_index);
    });
}

int st_dev_combine(st_ctx *c, const st_ttable *const *srcs, int32_t nsrc, const st_ttable *dst) {
    return guarded([&] {
        ST_ARG(c && srcs && nsrc > 0, "NULL argument");
        for (int i = 0; i < nsrc; ++i) check_ttable(srcs[i]);
        check_ttable(dst);
        use_device(c);
        combine_tdev(c, srcs, nsrc, dst);
    });
}

int st_dev_morton_order(st_ctx *c, const float *x, const float *y, const float *z, uint32_t *idx, uint64_t n) {
    return guarded([&] {
        ST_ARG(c && ((x && y && z && idx) || n == 0), "NULL argument");
        use_device(c);
        morton_order_dev(c, x, y, z, idx, n);
    });
}

int st_dev_pack_compressed(st_ctx *c, const st_table *t, const uint32_t *order, float *chunk, uint32_t *vertex,
                           uint8_t *sh) {
    return guarded([&] {
        ST_ARG(c && ((order && chunk && vertex) || t->n == 0), "NULL argument");
        check_table(t);
        use_device(c);
        pack_compressed_dev(c, t, order, chunk, vertex, sh);
    });
}

int st_dev_kmeans(st_ctx *c, const float *const *cols, int32_t d, uint64_t n, int32_t k, int32_t iters,
                  const double *draws, uint64_t ndraws, uint64_t *used, float *centroids, uint32_t *labels) {
    return guarded([&] {
        ST_ARG(c && cols && d > 0 && k > 0 && iters >= 0 && centroids && labels, "bad argument");
        ST_ARG(draws || ndraws == 0, "draws is NULL");
        use_device(c);
        begin_timing(c);
        uint64_t u = kmeans_dev(c, cols, d, n, k, iters, draws, ndraws, centroids, labels);
        end_timing(c);
        if (used) *used = u;
    });
}

int st_dev_cluster1d(st_ctx *c, const float *const *cols, int32_t ncols, uint64_t n, int32_t iters,
                     const double *draws, uint64_t ndraws, uint64_t *used, float *centroids, uint8_t *labels) {
    return guarded([&] {
        ST_ARG(c && cols && ncols > 0 && centroids && labels, "bad argument");
        use_device(c);
        begin_timing(c);
        uint64_t u = cluster1d_dev(c, cols, ncols, n, iters, draws, ndraws, centroids, labels);
        end_timing(c);
        if (used) *used = u;
    });
}

int st_dev_sog(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
               st_sog_meta *meta, const st_sog_textures *out) {
    return guarded([&] {
        ST_ARG(c && meta && out, "NULL argument");
        check_table(t);
        use_device(c);
        begin_timing(c);
        uint64_t u = sog_dev(c, t, iters, draws, ndraws, meta, out);
        end_timing(c);
        if (used) *used = u;
    });
}

int st_dev_sog_file(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                    st_sog_meta *meta, const st_sog_textures *out, int32_t fd, uint16_t dos_time, uint16_t dos_date,
                    uint64_t *size) {
    return guarded([&] {
        ST_ARG(c && meta && out && size && fd >= 0, "bad argument");
        check_table(t);
        use_device(c);
        begin_timing(c);
        uint64_t u = sog_file_dev(c, t, iters, draws, ndraws, meta, out, fd, dos_time, dos_date, size);
        end_timing(c);
        if (used) *used = u;
    });
}

// ---- multi-GPU building blocks ------------------------------------------------------
int st_dev_minmax(st_ctx *c, const float *const *cols, int32_t ncols, uint64_t n, double *lo, double *hi) {
    return guarded([&] {
        ST_ARG(c && cols && ncols > 0 && lo && hi, "bad argument");
        use_device(c);
        minmax_dev(c, cols, ncols, n, lo, hi);
    });
}

int st_dev_kmeans_prepare(st_ctx *c, const float *const *cols, int32_t d, uint64_t n) {
    return guarded([&] {
        ST_ARG(c && cols && d > 0 && n > 0, "bad argument");
        use_device(c);
        dist_prepare(c, cols, d, n);
    });
}

int st_dev_kmeans_assign(st_ctx *c, const float *const *cols, int32_t d, uint64_t n, int32_t k,
                         const float *centroids, uint32_t *labels) {
    return guarded([&] {
        ST_ARG(c && cols && d > 0 && n > 0 && k > 0 && centroids && labels, "bad argument");
        use_device(c);
        dist_assign(c, cols, d, n, k, centroids, labels);
    });
}

int st_dev_kmeans_init_rows(st_ctx *c, const double *draws, uint64_t ndraws, uint64_t n, int32_t k, uint32_t *rows,
                            uint64_t *used) {
    return guarded([&] {
        ST_ARG(c && (draws || ndraws == 0) && k > 0 && rows && used, "bad argument");
        use_device(c);
        kmeans_init_rows(c, draws, ndraws, n, k, rows, used);
    });
}

int st_dev_gather_rows(st_ctx *c, const float *const *cols, int32_t d, uint64_t n_local, uint64_t offset,
                       const uint32_t *rows, int32_t k, float *out) {
    return guarded([&] {
        ST_ARG(c && cols && d > 0 && k > 0 && rows && out, "bad argument");
        use_device(c);
        gather_owned_rows(c, cols, d, n_local, offset, rows, k, out);
    });
}

int st_dev_kmeans_partials(st_ctx *c, const float *const *cols, int32_t d, uint64_t n, int32_t nseg, int32_t k,
                           const uint32_t *labels, double *sums, double *sabs, int32_t *emin, uint32_t *counts) {
    return guarded([&] {
        ST_ARG(c && cols && d > 0 && n > 0 && k > 0 && labels && sums && sabs && emin && counts, "bad argument");
        use_device(c);
        dist_partials(c, cols, d, n, nseg, k, labels, sums, sabs, emin, counts);
    });
}

int st_dev_kmeans_seqsum(st_ctx *c, int32_t d, int32_t k, int32_t seg, const uint32_t *pairs, uint32_t npairs,
                         double *running, const int32_t *emin, const double *sabs) {
    return guarded([&] {
        ST_ARG(c && (npairs == 0 || (pairs && running && emin && sabs)), "bad argument");
        use_device(c);
        dist_seqsum(c, d, k, seg, pairs, npairs, running, emin, sabs);
    });
}

int st_dev_kmeans_finish(st_ctx *c, int32_t d, int32_t k, const double *sums, const double *sabs,
                         const int32_t *emin, const uint32_t *counts, float *centroids, uint32_t *pending,
                         uint32_t *npending) {
    return guarded([&] {
        ST_ARG(c && d > 0 && k > 0 && sums && sabs && emin && counts && centroids && pending && npending,
               "bad argument");
        use_device(c);
        *npending = dist_finish(c, d, k, sums, sabs, emin, counts, centroids, pending);
    });
}

int st_dev_kmeans_average(st_ctx *c, int32_t d, int32_t k, const uint32_t *pairs, uint32_t npairs,
                          const double *running, const uint32_t *counts, float *centroids) {
    return guarded([&] {
        ST_ARG(c && d > 0 && k > 0 && (npairs == 0 || (pairs && running)) && counts && centroids, "bad argument");
        use_device(c);
        dist_average(c, d, k, pairs, npairs, running, counts, centroids);
    });
}

int st_dev_cluster1d_codebook(st_ctx *c, const float *centroids, const uint32_t *labels, uint64_t total,
                              float *codebook256, uint8_t *labels8) {
    return guarded([&] {
        ST_ARG(c && centroids && codebook256 && (total == 0 || (labels && labels8)), "bad argument");
        use_device(c);
        codebook_dev(c, centroids, labels, total, codebook256, labels8);
    });
}

int st_dev_sog_scatter(st_ctx *c, const st_table *local, const uint32_t *pos, const double lo[3], const double hi[3],
                       const uint8_t *scale_labels, const uint8_t *color_labels, const uint32_t *shn_labels,
                       st_sog_meta *meta, const st_sog_textures *out) {
    return guarded([&] {
        ST_ARG(c && (pos || local->n == 0) && lo && hi && meta && out, "bad argument");
        check_table(local);
        use_device(c);
        sog_scatter_dev(c, local, pos, lo, hi, scale_labels, color_labels, shn_labels, meta, out);
    });
}

int st_dev_sog_shn_centroids(st_ctx *c, const uint8_t *codebook_labels, int32_t sh_coeffs, int32_t palette,
                             uint8_t *out) {
    return guarded([&] {
        ST_ARG(c && codebook_labels && sh_coeffs > 0 && palette > 0 && out, "bad argument");
        use_device(c);
        shn_centroids_dev(c, codebook_labels, sh_coeffs, palette, out);
    });
}

}  // extern "C"
