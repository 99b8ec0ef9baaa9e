// st_multi.hip -- writeSog over a table whose rows are sharded across GPUs,
// native: the k-means iterations, the centroid-sum exchange and the texel gather run in the
// library, over RCCL (xGMI) between the ranks.
//
// A rank is one (device context, host thread).  Rows are sharded in contiguous ranges in rank
// order; the global table is the concatenation of the shards (for config 5 the concatenation
// of the input files: combine(), index.ts:158-210).  Results equal the single-device writeSog
// of the global table bit for bit:
//   * k-means (k-means.ts:137-201): assign is row-local.  calcAverage adds each cluster's
//     members in ascending global point order in f64; every rank computes exact partials
//     (sum, sum|x|, smallest ulp exponent, count) and where sum|x| < 2^(emin+53) the all-reduced
//     sum is that sum (every partial sum is exact); the remaining (cluster, dim) pairs replay the
//     sequential sum, the running value handed from segment to segment in global order.
//     Math.random: every rank holds the same draws and consumes them identically; a drawn row
//     is supplied by its owner (bit patterns, integer SUM all-reduce).  That is the SH palette's
//     k-means; the two cluster1d (scales, colours: 28 B of columns per row, 20 latency-bound
//     iterations) run over the gathered columns as on one device, the scales on rank 0 and the
//     colours on rank 1, and every rank takes the draws they consumed from those two.
//   * Morton order (ordering.ts:4-110) is global: rank 0 gathers x/y/z and orders the whole
//     table; every rank writes the texels of its rows in row order and rank 0 places them at
//     their Morton positions.  Both run beside the k-means: a side host thread per rank moves
//     the rows over a second channel (Coll::side, an ncclCommSplit) on its side stream, so only
//     the shN labels' gather and placement follow the SH k-means.
//
// Transports (Coll): RCCL (one process per GPU via a unique id, or one process driving
// several GPUs via ncclCommInitAll), and a host-staged exchange between threads of one process
// (several ranks on one GPU: the multi-rank tests on a one-GPU box).
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <thread>

#include "st_coll.h"
#include "st_internal.h"
#include "st_kmeans.h"
#include "st_webp.h"
#include "st_rccl.h"

// every RCCL entry point through the run-time binding (st_rccl.h: one RCCL file for both hosts)
#define ncclGetErrorString (::st::rccl().GetErrorString)
#define ncclGetUniqueId (::st::rccl().GetUniqueId)
#define ncclCommInitRank (::st::rccl().CommInitRank)
#define ncclCommInitAll (::st::rccl().CommInitAll)
#define ncclCommSplit (::st::rccl().CommSplit)
#define ncclCommDestroy (::st::rccl().CommDestroy)
#define ncclCommAbort (::st::rccl().CommAbort)
#define ncclCommCount (::st::rccl().CommCount)
#define ncclAllReduce (::st::rccl().AllReduce)
#define ncclBroadcast (::st::rccl().Broadcast)
#define ncclAllGather (::st::rccl().AllGather)
#define ncclSend (::st::rccl().Send)
#define ncclRecv (::st::rccl().Recv)
#define ncclGroupStart (::st::rccl().GroupStart)
#define ncclGroupEnd (::st::rccl().GroupEnd)

namespace st {

int palette_of(uint64_t n);

#define ST_NCCL(expr)                                                                             \
    do {                                                                                          \
        ncclResult_t _r = (expr);                                                                 \
        if (_r != ncclSuccess)                                                                    \
            throw ::st::Error(ST_ERR_INTERNAL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

struct RcclColl : Coll {
    // `comm` is written once, before any rank thread runs; an abort only flips `dead` (atomic)
    // and aborts the communicator, so a rank thread never reads a pointer another thread writes.
    // A call that starts after the abort throws; one already inside RCCL returns the abort.
    ncclComm_t comm = nullptr;
    bool own = true;
    std::atomic<bool> dead{false};
    std::mutex side_mu;
    std::unique_ptr<RcclColl> side_;  // ncclCommSplit of comm
    bool enqueues() const override { return true; }
    ~RcclColl() override {
        side_.reset();
        if (comm && own && !dead.load()) ncclCommDestroy(comm);
    }
    Coll *side() override {
        live();
        std::lock_guard<std::mutex> lk(side_mu);
        if (!side_) {
            auto sc = std::make_unique<RcclColl>();
            ST_NCCL(ncclCommSplit(comm, 0, rank, &sc->comm, nullptr));
            sc->rank = rank;
            sc->world = world;
            side_ = std::move(sc);
        }
        return side_.get();
    }
    void live() const {
        if (dead.load()) throw Error(ST_ERR_INTERNAL, "multi-GPU: another rank failed");
    }
    static ncclDataType_t nt(Dt d) { return d == Dt::F64 ? ncclFloat64 : ncclInt32; }
    static ncclRedOp_t no(Op o) { return o == Op::Sum ? ncclSum : ncclMin; }
    void allreduce(void *buf, size_t count, Dt dt, Op op, hipStream_t s) override {
        live();
        if (world > 1 && count) ST_NCCL(ncclAllReduce(buf, buf, count, nt(dt), no(op), comm, s));
    }
    void broadcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        live();
        if (world > 1 && bytes) ST_NCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm, s));
    }
    void allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        live();
        if (world == 1) {
            if (bytes && recv != send) ST_HIP(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
            return;
        }
        ST_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, comm, s));
    }
    void gatherv(const void *send, size_t mybytes, void *recv, const std::vector<size_t> &bytes,
                 const std::vector<size_t> &displ, int root, hipStream_t s) override {
        live();
        if (rank == root && mybytes)
            ST_HIP(hipMemcpyAsync(static_cast<char *>(recv) + displ[rank], send, mybytes, hipMemcpyDeviceToDevice, s));
        if (world == 1) return;
        ST_NCCL(ncclGroupStart());
        if (rank == root) {
            for (int r = 0; r < world; ++r)
                if (r != root && bytes[r]) ST_NCCL(ncclRecv(static_cast<char *>(recv) + displ[r], bytes[r], ncclUint8, r, comm, s));
        } else if (mybytes) {
            ST_NCCL(ncclSend(send, mybytes, ncclUint8, root, comm, s));
        }
        ST_NCCL(ncclGroupEnd());
    }
    void gatherv_many(const std::vector<Gather> &gs, const std::vector<size_t> &bytes,
                      const std::vector<size_t> &displ, hipStream_t s) override {
        live();
        for (const Gather &g : gs)
            if (rank == g.root && g.mybytes)
                ST_HIP(hipMemcpyAsync(static_cast<char *>(g.recv) + displ[rank], g.send, g.mybytes,
                                      hipMemcpyDeviceToDevice, s));
        if (world == 1) return;
        ST_NCCL(ncclGroupStart());
        for (const Gather &g : gs) {
            if (rank == g.root) {
                for (int r = 0; r < world; ++r)
                    if (r != g.root && bytes[r])
                        ST_NCCL(ncclRecv(static_cast<char *>(g.recv) + displ[r], bytes[r], ncclUint8, r, comm, s));
            } else if (g.mybytes) {
                ST_NCCL(ncclSend(g.send, g.mybytes, ncclUint8, g.root, comm, s));
            }
        }
        ST_NCCL(ncclGroupEnd());
    }
    void sendrecv(void *buf, size_t bytes, int from, int to, hipStream_t s) override {
        live();
        if (world == 1 || from == to || !bytes || (rank != from && rank != to)) return;
        if (rank == from) ST_NCCL(ncclSend(buf, bytes, ncclUint8, to, comm, s));
        else ST_NCCL(ncclRecv(buf, bytes, ncclUint8, from, comm, s));
    }
    void abort() override {
        {
            std::lock_guard<std::mutex> lk(side_mu);
            if (side_) side_->abort();
        }
        if (!dead.exchange(true) && comm) ncclCommAbort(comm);
    }
    int count() const {
        int n = 0;
        ST_NCCL(ncclCommCount(comm, &n));
        return n;
    }
};

// host-staged exchange between the threads of one process (any number of ranks per GPU)
struct HostHub {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool aborted = false;
    std::vector<std::vector<char>> slot;
    std::shared_ptr<HostHub> side;  // the second channel's hub (made by the first rank asking)
    explicit HostHub(int w) : world(w), slot(w) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) throw Error(ST_ERR_INTERNAL, "multi-GPU: another rank failed");
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || aborted; });
        }
        if (aborted) throw Error(ST_ERR_INTERNAL, "multi-GPU: another rank failed");
    }
    void abort() {
        std::shared_ptr<HostHub> sd;
        {
            std::lock_guard<std::mutex> lk(mu);
            aborted = true;
            cv.notify_all();
            sd = side;
        }
        if (sd) sd->abort();
    }
    std::shared_ptr<HostHub> side_hub() {
        std::lock_guard<std::mutex> lk(mu);
        if (!side) side = std::make_shared<HostHub>(world);
        if (aborted) side->abort();
        return side;
    }
};

struct HostColl : Coll {
    std::shared_ptr<HostHub> hub;
    std::unique_ptr<HostColl> side_;
    bool enqueues() const override { return false; }
    Coll *side() override {
        if (!side_) {
            auto sc = std::make_unique<HostColl>();
            sc->hub = hub->side_hub();
            sc->rank = rank;
            sc->world = world;
            side_ = std::move(sc);
        }
        return side_.get();
    }
    void put(const void *dev, size_t bytes, hipStream_t s) {
        auto &v = hub->slot[rank];
        v.resize(bytes);
        if (bytes) ST_HIP(hipMemcpyAsync(v.data(), dev, bytes, hipMemcpyDeviceToHost, s));
        ST_HIP(hipStreamSynchronize(s));
    }
    void allreduce(void *buf, size_t count, Dt dt, Op op, hipStream_t s) override {
        const size_t es = dt == Dt::F64 ? 8 : 4;
        put(buf, count * es, s);
        hub->barrier();
        std::vector<char> acc(hub->slot[0]);
        for (int r = 1; r < world; ++r) {
            const char *src = hub->slot[r].data();
            for (size_t i = 0; i < count; ++i) {
                if (dt == Dt::F64) {
                    double a, b;
                    std::memcpy(&a, acc.data() + 8 * i, 8);
                    std::memcpy(&b, src + 8 * i, 8);
                    a = op == Op::Sum ? a + b : std::min(a, b);
                    std::memcpy(acc.data() + 8 * i, &a, 8);
                } else {
                    int32_t a, b;
                    std::memcpy(&a, acc.data() + 4 * i, 4);
                    std::memcpy(&b, src + 4 * i, 4);
                    a = op == Op::Sum ? (int32_t)((uint32_t)a + (uint32_t)b) : std::min(a, b);
                    std::memcpy(acc.data() + 4 * i, &a, 4);
                }
            }
        }
        hub->barrier();  // every rank has read the slots
        if (count) ST_HIP(hipMemcpyAsync(buf, acc.data(), count * es, hipMemcpyHostToDevice, s));
        ST_HIP(hipStreamSynchronize(s));
    }
    void broadcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        if (rank == root) put(buf, bytes, s);
        hub->barrier();
        std::vector<char> v;
        if (rank != root) v = hub->slot[root];
        hub->barrier();
        if (rank != root && bytes) {
            ST_HIP(hipMemcpyAsync(buf, v.data(), bytes, hipMemcpyHostToDevice, s));
            ST_HIP(hipStreamSynchronize(s));
        }
    }
    void allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        put(send, bytes, s);
        hub->barrier();
        std::vector<char> all(bytes * world);
        for (int r = 0; r < world; ++r)
            if (bytes) std::memcpy(all.data() + bytes * r, hub->slot[r].data(), bytes);
        hub->barrier();
        if (bytes) ST_HIP(hipMemcpyAsync(recv, all.data(), bytes * world, hipMemcpyHostToDevice, s));
        ST_HIP(hipStreamSynchronize(s));
    }
    void gatherv(const void *send, size_t mybytes, void *recv, const std::vector<size_t> &bytes,
                 const std::vector<size_t> &displ, int root, hipStream_t s) override {
        put(send, mybytes, s);
        hub->barrier();
        if (rank == root) {
            for (int r = 0; r < world; ++r)
                if (bytes[r])
                    ST_HIP(hipMemcpyAsync(static_cast<char *>(recv) + displ[r], hub->slot[r].data(), bytes[r],
                                          hipMemcpyHostToDevice, s));
            ST_HIP(hipStreamSynchronize(s));
        }
        hub->barrier();
    }
    void sendrecv(void *buf, size_t bytes, int from, int to, hipStream_t s) override {
        if (rank == from) put(buf, bytes, s);
        hub->barrier();
        if (rank == to && from != to && bytes) {
            ST_HIP(hipMemcpyAsync(buf, hub->slot[from].data(), bytes, hipMemcpyHostToDevice, s));
            ST_HIP(hipStreamSynchronize(s));
        }
        hub->barrier();
    }
    void abort() override { hub->abort(); }
};

// ---------------------------------------------------------------------------
namespace {

using namespace km;

// out[c][i] = bits of pts[c][local[i]] for the slots this rank supplies (local[i] != ~0u), 0 elsewhere
__global__ __launch_bounds__(256) void k_pick_bits(const float *const *pts, int d, const uint32_t *local, int m,
                                                   uint32_t *out) {
    const int total = d * m;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int c = t / m, i = t % m;
        const uint32_t li = local[i];
        out[t] = li == ~0u ? 0u : __builtin_bit_cast(uint32_t, pts[c][li]);
    }
}

// cen[c][cl[i]] = vals[c][i]
__global__ __launch_bounds__(256) void k_put_rows(const float *vals, int d, int m, const uint32_t *cl, int k,
                                                  float *cen) {
    const int total = d * m;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int c = t / m, i = t % m;
        cen[(uint64_t)c * k + cl[i]] = vals[t];
    }
}

// fold the per-segment partials [nseg][d][k] into SAC = [sum (d*k) | sum|x| (d*k) | count (k)]
// (f64: counts are exact below 2^53) and E = min emin [d*k]
__global__ __launch_bounds__(256) void k_counts_f64(const uint32_t *counts, int k, double *out) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x) out[i] = (double)counts[i];
}

__global__ __launch_bounds__(256) void k_fold_partials(const double *sums, const double *sabs, const int32_t *emin,
                                                       const uint32_t *counts, int nseg, int d, int k, double *sac,
                                                       int32_t *e) {
    const uint32_t dk = (uint32_t)d * k;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < dk + (uint32_t)k; t += gridDim.x * blockDim.x) {
        if (t < dk) {
            double s = 0, a = 0;
            int32_t m = 1 << 20;
            for (int g = 0; g < nseg; ++g) {
                s += sums[(uint64_t)g * dk + t];
                a += sabs[(uint64_t)g * dk + t];
                m = min(m, emin[(uint64_t)g * dk + t]);
            }
            sac[t] = s;
            sac[dk + t] = a;
            e[t] = m;
        } else {
            const uint32_t cl = t - dk;
            double cnt = 0;
            for (int g = 0; g < nseg; ++g) cnt += (double)counts[(uint64_t)g * k + cl];
            sac[2 * dk + cl] = cnt;
        }
    }
}

__global__ __launch_bounds__(256) void k_counts_u32(const double *c, int k, uint32_t *out) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < k; t += gridDim.x * blockDim.x) out[t] = (uint32_t)c[t];
}

// texture of the global table: tex[pos[g]] = texels[g] (4 bytes per row)
__global__ __launch_bounds__(256) void k_place(const uint32_t *texels, const uint32_t *pos, uint64_t n, uint32_t *tex) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x)
        tex[pos[g]] = texels[g];
}

__global__ __launch_bounds__(256) void k_invert_u32(const uint32_t *idx, uint64_t n, uint32_t *pos) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        pos[idx[i]] = (uint32_t)i;
}

struct Shard {
    int rank = 0, world = 1;
    std::vector<uint64_t> counts, offsets;
    uint64_t n = 0, off = 0, N = 0;
    int owner(uint64_t row) const {
        for (int r = 0; r < world; ++r)
            if (row >= offsets[r] && row < offsets[r] + counts[r]) return r;
        return -1;
    }
};

Shard make_shard(st_ctx *c, Coll &co, uint64_t n_local) {
    Shard s;
    s.rank = co.rank;
    s.world = co.world;
    auto *dn = wsT<uint64_t>(c, "mg.n", 1);
    auto *dall = wsT<uint64_t>(c, "mg.nall", (size_t)co.world);
    ST_HIP(hipMemcpyAsync(dn, &n_local, 8, hipMemcpyHostToDevice, c->stream));
    co.allgather(dn, dall, 8, c->stream);
    s.counts.resize(co.world);
    ST_HIP(hipMemcpyAsync(s.counts.data(), dall, 8 * co.world, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    s.offsets.resize(co.world);
    uint64_t acc = 0;
    for (int r = 0; r < co.world; ++r) {
        s.offsets[r] = acc;
        acc += s.counts[r];
    }
    s.N = acc;
    s.n = n_local;
    s.off = s.offsets[co.rank];
    return s;
}

// the k-means point set of one rank: d columns (concat = false), or cluster1d's 1-D
// concatenation of `ncols` columns (global point g = column g / N, row g % N)
struct Points {
    const Shard *sh;
    bool concat;
    int d, nseg;
    uint64_t n, N;
    std::vector<const float *> pts;
    // (owner, local index) of global point g
    std::pair<int, uint64_t> locate(uint64_t g) const {
        if (!concat) {
            const int r = sh->owner(g);
            return {r, r < 0 ? 0 : g - sh->offsets[r]};
        }
        const uint64_t col = g / sh->N, row = g % sh->N;
        const int r = sh->owner(row);
        return {r, r < 0 ? 0 : col * sh->counts[r] + (row - sh->offsets[r])};
    }
};

// values of global points `rows` as centroid columns at slots `cl` of cen (every rank)
void supply_rows(st_ctx *c, Coll &co, const Points &P, const std::vector<uint64_t> &rows,
                 const std::vector<uint32_t> &cl, int k, float *cen) {
    const int m = (int)rows.size();
    if (!m) return;
    std::vector<uint32_t> local(m, ~0u);
    for (int i = 0; i < m; ++i) {
        auto o = P.locate(rows[i]);
        ST_REQUIRE(o.first >= 0, ST_ERR_ARG, "kmeans: drawn row outside the table");
        if (o.first == co.rank) local[i] = (uint32_t)o.second;
    }
    auto *dlocal = wsT<uint32_t>(c, "mg.local", m);
    auto *dcl = wsT<uint32_t>(c, "mg.cl", m);
    auto *vals = wsT<uint32_t>(c, "mg.vals", (size_t)m * P.d);
    auto **dpts = wsT<const float *>(c, "mg.pts", (size_t)P.d);
    ST_HIP(hipMemcpyAsync(dlocal, local.data(), 4 * m, hipMemcpyHostToDevice, c->stream));
    ST_HIP(hipMemcpyAsync(dcl, cl.data(), 4 * m, hipMemcpyHostToDevice, c->stream));
    ST_HIP(hipMemcpyAsync(dpts, P.pts.data(), sizeof(float *) * P.d, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_pick_bits, dim3(grid_for((uint64_t)m * P.d, 256, 4096)), dim3(256), 0, c->stream, dpts, P.d,
                       dlocal, m, vals);
    ST_LAUNCH_CHECK();
    co.allreduce(vals, (size_t)m * P.d, Dt::I32, Op::Sum, c->stream);  // owners' bit patterns, 0 elsewhere
    hipLaunchKernelGGL(k_put_rows, dim3(grid_for((uint64_t)m * P.d, 256, 4096)), dim3(256), 0, c->stream,
                       (const float *)vals, P.d, m, dcl, k, cen);
    ST_LAUNCH_CHECK();
    ST_HIP(hipStreamSynchronize(c->stream));  // local / cl are released on return
}

// kmeans over the global point set (k-means.ts:137-201); cen [d][k] (device), labels (local, device)
uint64_t kmeans_sharded(st_ctx *c, Coll &co, const Points &P, int k, int iters, const double *draws,
                        uint64_t ndraws, float *cen, uint32_t *labels, const char *tag) {
    const int d = P.d;
    ST_REQUIRE(P.N >= (uint64_t)k, ST_ERR_UNSUPPORTED, "multi-GPU kmeans with fewer points than clusters");
    if (P.n) dist_prepare(c, P.pts.data(), d, P.n);
    uint64_t cursor = 0;
    const uint64_t dk = (uint64_t)d * k;
    if (d == 1) {
        // initializeCentroids1D (k-means.ts:23-39) over the global min / max
        double lo, hi;
        minmax_dev(c, P.pts.data(), 1, P.n, &lo, &hi);
        auto *mm = wsT<double>(c, "mg.mm", 2);
        double h2[2] = {lo, -hi};
        ST_HIP(hipMemcpyAsync(mm, h2, 16, hipMemcpyHostToDevice, c->stream));
        co.allreduce(mm, 2, Dt::F64, Op::Min, c->stream);
        ST_HIP(hipMemcpyAsync(h2, mm, 16, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        const double m = h2[0], M = -h2[1];
        std::vector<float> init(k);
        for (int i = 0; i < k; ++i) init[i] = (float)(m + (M - m) * i / (k - 1));
        ST_HIP(hipMemcpyAsync(cen, init.data(), 4 * k, hipMemcpyHostToDevice, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
    } else {
        // initializeCentroids (k-means.ts:8-20): the same k global rows on every rank; owners
        // supply the values, an integer SUM of the bit patterns assembles them exactly
        auto *rows = wsT<uint32_t>(c, "mg.rows", (size_t)k);
        uint64_t used = 0;
        kmeans_init_rows(c, draws, ndraws, P.N, k, rows, &used);
        cursor += used;
        gather_owned_rows(c, P.pts.data(), d, P.n, P.sh->off, rows, k, cen);
        co.allreduce(cen, dk, Dt::I32, Op::Sum, c->stream);
    }
    const std::string t(tag);
    if (d > 1) c->kn_stats = st_ctx::KnStats{};
    auto *sac = wsT<double>(c, t + ".sac", 2 * dk + k);
    auto *E = wsT<int32_t>(c, t + ".e", dk);
    auto *C = wsT<uint32_t>(c, t + ".c", (size_t)k);
    auto *sums = wsT<double>(c, t + ".sums", P.nseg * dk);
    auto *sabs = wsT<double>(c, t + ".sabs", P.nseg * dk);
    auto *emin = wsT<int32_t>(c, t + ".emin", P.nseg * dk);
    auto *counts = wsT<uint32_t>(c, t + ".counts", (size_t)P.nseg * k);
    auto *pending = wsT<uint32_t>(c, t + ".pend", dk);
    auto *running = wsT<double>(c, t + ".run", dk);
    // the counts come back with dist_finish's readback (one stream sync per iteration)
    auto *hC = static_cast<uint32_t *>(pinned_slot(c, t + ".hC", 4 * (size_t)k));
    const size_t cbytes = 4 * dk;
    // the shard's column pointers on the device, uploaded once for the N-D iterations
    auto **dpts = wsT<const float *>(c, t + ".dpts", (size_t)d);
    if (P.n && d > 1)
        ST_HIP(hipMemcpyAsync(dpts, P.pts.data(), sizeof(float *) * d, hipMemcpyHostToDevice, c->stream));
    for (int it = 0; it < iters; ++it) {
        bool folded = false;  // the partials are already in sac / E
        if (c->verify && d > 1 && it == iters - 1)  // st_ctx_set_verify: the last assign's centroids
            ST_HIP(hipMemcpyAsync(ws(c, "verify.prev", cbytes), cen, cbytes, hipMemcpyDeviceToDevice, c->stream));
        if (P.n && d == 1 && k <= 256 && !getenv("ST_K1_SORT")) {
            dist_assign_partials1d(c, P.pts[0], P.n, P.nseg, k, cen, labels, sums, sabs, emin, counts);
        } else if (P.n && d > 1 && P.nseg == 1 && !getenv("ST_ND_SORT")) {
            // the fused fix-up's partials (ST_ND_SORT=1: the member sort), written straight into
            // the all-reduce's layout (one segment: nothing to fold but the counts)
            folded = dist_assign_partials_nd(c, dpts, d, P.n, k, cen, labels, sac, sac + dk, E, counts);
            if (!folded) dist_partials(c, P.pts.data(), d, P.n, P.nseg, k, labels, sums, sabs, emin, counts);
        } else if (P.n) {
            dist_assign(c, P.pts.data(), d, P.n, k, cen, labels);
            dist_partials(c, P.pts.data(), d, P.n, P.nseg, k, labels, sums, sabs, emin, counts);
        } else {  // empty shard: neutral partials
            ST_HIP(hipMemsetAsync(sums, 0, 8 * P.nseg * dk, c->stream));
            ST_HIP(hipMemsetAsync(sabs, 0, 8 * P.nseg * dk, c->stream));
            ST_HIP(hipMemsetD32Async(emin, 1 << 20, P.nseg * dk, c->stream));
            ST_HIP(hipMemsetAsync(counts, 0, 4 * (size_t)P.nseg * k, c->stream));
        }
        if (folded)
            hipLaunchKernelGGL(k_counts_f64, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, counts, k,
                               sac + 2 * dk);
        else
            hipLaunchKernelGGL(k_fold_partials, dim3(grid_for(dk + k, 256, 4096)), dim3(256), 0, c->stream, sums,
                               sabs, emin, counts, P.nseg, d, k, sac, E);
        ST_LAUNCH_CHECK();
        co.allreduce(sac, 2 * dk + k, Dt::F64, Op::Sum, c->stream);
        co.allreduce(E, dk, Dt::I32, Op::Min, c->stream);
        hipLaunchKernelGGL(k_counts_u32, dim3(grid_for(k, 256, 1024)), dim3(256), 0, c->stream, sac + 2 * dk, k, C);
        ST_LAUNCH_CHECK();
        ST_HIP(hipMemcpyAsync(hC, C, 4 * (size_t)k, hipMemcpyDeviceToHost, c->stream));
        const uint32_t np = dist_finish(c, d, k, sac, sac + dk, E, C, cen, pending);
        if (np) {
            // the sequential f64 chain of each pending (cluster, dim): segments in global order
            // the sequential f64 chain of each pending (cluster, dim): segments in global order, the
            // running values handed from owner to owner (point to point), then to every rank
            ST_HIP(hipMemsetAsync(running, 0, 8 * (size_t)np, c->stream));
            int prev = -1;
            for (int seg = 0; seg < P.nseg; ++seg)
                for (int r = 0; r < co.world; ++r) {
                    if (prev >= 0) co.sendrecv(running, 8 * (size_t)np, prev, r, c->stream);
                    if (r == co.rank && P.n) dist_seqsum(c, d, k, seg, pending, np, running, E, sac + dk);
                    prev = r;
                }
            co.broadcast(running, 8 * (size_t)np, prev, c->stream);
            dist_average(c, d, k, pending, np, running, C, cen);
        }
        // re-seed the empty clusters (k-means.ts:174-178): ascending clusters, one draw each (hC
        // arrived with dist_finish's sync)
        std::vector<uint64_t> rows;
        std::vector<uint32_t> cls;
        for (int i = 0; i < k; ++i) {
            if (hC[i]) continue;
            ST_REQUIRE(cursor < ndraws, ST_ERR_DRAWS, "kmeans: Math.random draws exhausted while re-seeding");
            const double dr = draws[cursor++];
            ST_REQUIRE(dr >= 0.0 && dr < 1.0, ST_ERR_ARG, "kmeans: a re-seed draw outside [0, 1)");
            rows.push_back((uint64_t)std::floor(dr * (double)P.N));
            cls.push_back((uint32_t)i);
        }
        supply_rows(c, co, P, rows, cls, k, cen);
    }
    if (c->verify && d > 1 && iters > 0) {  // final centroids (replicated) and this rank's labels
        ST_HIP(hipMemcpyAsync(ws(c, "verify.cen", cbytes), cen, cbytes, hipMemcpyDeviceToDevice, c->stream));
        if (P.n)
            ST_HIP(hipMemcpyAsync(ws(c, "verify.labels", P.n * 4), labels, P.n * 4, hipMemcpyDeviceToDevice,
                                  c->stream));
        c->vf_d = d;
        c->vf_k = k;
        c->vf_n = P.n;
    }
    if (d > 1) kn_stats_publish(c);  // this rank's points
    return cursor;
}

// the rank's rows of the member columns (the combine of its local tables: every column of the
// union, absent ones zero-filled, index.ts:158-210); band from the union over every rank
struct LocalTable {
    std::vector<std::string> names;
    std::vector<const char *> cnames;
    std::vector<float *> cols;
    st_table t{};
    int C = 0;
};

const char *kMembers[14] = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "f_dc_0",
                            "f_dc_1", "f_dc_2", "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};

LocalTable combine_local(st_ctx *c, Coll &co, const st_table *const *tabs, int ntab) {
    LocalTable L;
    // f_rest presence over every rank's tables (union of names) -> the band rule
    int32_t present[46] = {0};
    for (int t = 0; t < ntab; ++t)
        for (int i = 0; i < 45; ++i) {
            char nm[32];
            snprintf(nm, sizeof nm, "f_rest_%d", i);
            if (find_col(tabs[t], nm) >= 0) present[i] = 1;
        }
    for (int i = 0; i < 45; ++i) present[i] = -present[i];  // MIN of the negation = OR
    auto *dp = wsT<int32_t>(c, "mg.present", 46);
    ST_HIP(hipMemcpyAsync(dp, present, 4 * 45, hipMemcpyHostToDevice, c->stream));
    co.allreduce(dp, 45, Dt::I32, Op::Min, c->stream);
    ST_HIP(hipMemcpyAsync(present, dp, 4 * 45, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    int miss = -1;
    for (int i = 0; i < 45 && miss < 0; ++i)
        if (!present[i]) miss = i;
    L.C = miss == 9 ? 3 : miss == 24 ? 8 : miss == -1 ? 15 : 0;  // write-sog.ts:296
    for (auto *m : kMembers) L.names.push_back(m);
    for (int i = 0; i < 3 * L.C; ++i) L.names.push_back("f_rest_" + std::to_string(i));
    uint64_t n = 0;
    for (int t = 0; t < ntab; ++t) n += tabs[t]->n;
    for (size_t j = 0; j < L.names.size(); ++j) {
        // one table with the column: use it in place; otherwise concatenate (zero where absent)
        int only = -1, have = 0;
        for (int t = 0; t < ntab; ++t)
            if (tabs[t]->n && find_col(tabs[t], L.names[j].c_str()) >= 0) {
                ++have;
                only = t;
            }
        float *col;
        if (ntab == 1 && have == 1) {
            col = tabs[only]->cols[find_col(tabs[only], L.names[j].c_str())];
        } else {
            col = wsT<float>(c, "mg.comb." + L.names[j], n);
            uint64_t off = 0;
            for (int t = 0; t < ntab; ++t) {
                const int ci = find_col(tabs[t], L.names[j].c_str());
                if (tabs[t]->n) {
                    if (ci >= 0)
                        ST_HIP(hipMemcpyAsync(col + off, tabs[t]->cols[ci], 4 * tabs[t]->n, hipMemcpyDeviceToDevice,
                                              c->stream));
                    else
                        ST_HIP(hipMemsetAsync(col + off, 0, 4 * tabs[t]->n, c->stream));
                }
                off += tabs[t]->n;
            }
        }
        L.cols.push_back(col);
    }
    for (auto &s : L.names) L.cnames.push_back(s.c_str());
    L.t.n = n;
    L.t.ncol = (int32_t)L.names.size();
    L.t.names = L.cnames.data();
    L.t.cols = L.cols.data();
    return L;
}

// the events one sharded writeSog orders its streams with
struct Events {
    hipEvent_t e[6] = {};
    Events() {
        for (auto &x : e) ST_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    }
    ~Events() {
        for (auto x : e)
            if (x) (void)hipEventDestroy(x);
    }
    hipEvent_t operator[](int i) const { return e[i]; }
};

// a rank's side worker: one host thread runs the pushed tasks in order.  The first failure
// aborts both channels (the peers must not wait for this rank) and the remaining tasks are
// skipped; drain() waits for the tasks and rethrows it.  Destroyed without drain() (this rank's
// main thread failed), it aborts both channels first, so a task blocked in an exchange returns.
struct SideWorker {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    bool stop = false, drained = false;
    std::exception_ptr err;
    Coll *a, *b;
    std::thread th;
    // ST_FAULT_SIDE_DELAY_MS=<ms> (fault injection, tests): a random delay before each task, so the
    // side channel's calls interleave differently with the main thread's
    int delay_ms = 0;
    std::minstd_rand rng{12345};
    SideWorker(int device, Coll *main, Coll *side) : a(main), b(side) {
        if (const char *d = getenv("ST_FAULT_SIDE_DELAY_MS")) delay_ms = std::max(0, atoi(d));
        rng.seed(12345u + (unsigned)main->rank * 7919u);
        th = std::thread([this, device] {
            bool dev_ok = hipSetDevice(device) == hipSuccess;
            for (;;) {
                std::function<void()> f;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || !q.empty(); });
                    if (q.empty()) return;
                    f = std::move(q.front());
                    q.pop_front();
                }
                if (err) continue;
                try {
                    ST_REQUIRE(dev_ok, ST_ERR_HIP, "side worker: hipSetDevice failed");
                    if (delay_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(rng() % (delay_ms + 1)));
                    f();
                } catch (...) {
                    err = std::current_exception();
                    a->abort();
                    if (b != a) b->abort();
                }
            }
        });
    }
    void push(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(f));
        }
        cv.notify_all();
    }
    void drain() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();
        drained = true;
        if (err) std::rethrow_exception(err);
    }
    ~SideWorker() {
        if (!drained) {
            a->abort();
            if (b != a) b->abort();
            std::lock_guard<std::mutex> lk(mu);
            q.clear();
            stop = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();
    }
};

}  // namespace

// writeSog's textures + meta (write-sog.ts:110-370) of the global table, on rank 0's device
// (`out`/`meta` are read on rank 0 only).  Returns the draws consumed.
static uint64_t sog_sharded_rank(st_ctx *c, Coll &co, const st_table *const *tabs, int ntab, int iters,
                                 const double *draws, uint64_t ndraws, st_sog_meta *meta, const st_sog_textures *out,
                                 uint64_t *n_global) {
    use_device(c);
    LocalTable L = combine_local(c, co, tabs, ntab);
    const st_table *t = &L.t;
    const Shard sh = make_shard(c, co, t->n);
    if (const char *f = getenv("ST_FAULT_RANK"))  // fault injection (tests): this rank fails here,
        ST_REQUIRE(atoi(f) != co.rank, ST_ERR_INTERNAL, "ST_FAULT_RANK: injected failure");  // the others wait in a collective
    const uint64_t N = sh.N;
    if (n_global) *n_global = N;
    ST_REQUIRE(N > 0, ST_ERR_ARG, "sog: empty table");
    ST_REQUIRE(N < (1ull << 31), ST_ERR_ARG, "sog: the table must have < 2^31 rows");
    const int C = L.C;
    int32_t W, H, pal, cw, chh;
    st_sog_geometry(N, C, &W, &H, &pal, &cw, &chh);
    const uint64_t texels = (uint64_t)W * H;
    const bool root = co.rank == 0;
    if (root) {
        *meta = st_sog_meta{};
        meta->width = W;
        meta->height = H;
        for (uint8_t *p : {out->means_l, out->means_u, out->quats, out->scales, out->sh0})
            ST_REQUIRE(p, ST_ERR_ARG, "sog: texture output is NULL");
        if (C) ST_REQUIRE(out->shn_centroids && out->shn_labels, ST_ERR_ARG, "sog: shN texture outputs are NULL");
    }
    const float *m[14];
    for (int i = 0; i < 14; ++i) m[i] = t->cols[i];
    static const char *texn[6] = {"means_l", "means_u", "quats", "scales", "sh0", "shN_labels"};
    const int ntex = C ? 6 : 5;

    // The global Morton order and the texel placement on rank 0 leave the critical path: x/y/z
    // and the first five textures move over the side channel (Coll::side) on the side stream, and
    // rank 0 orders the table and places those texels on its side context from a worker thread,
    // all beside the k-means on this thread.  Only the shN labels (known after the SH k-means) are
    // gathered and placed after it.  Who issues the side channel's calls (Coll::enqueues):
    //   * RCCL: this thread, at fixed points of its program (before the cluster1d k-means and
    //     before the SH k-means), so every rank enqueues the two communicators' collectives in the
    //     same order -- blocking collective kernels that share a hardware queue can then never
    //     wait on each other in opposite orders on two ranks; the worker only runs rank 0's
    //     Morton order and placement (no collective);
    //   * host-staged transports (calls return when the bytes have moved): the worker, in order;
    //     their channels' hubs are independent.
    // ST_SIDE_CHANNEL=0 (the launcher's fallback) moves all of it onto the main channel, stream
    // and thread, in the same program order.
    std::vector<size_t> bytes(co.world), displ(co.world);
    for (int r = 0; r < co.world; ++r) {
        bytes[r] = 4 * sh.counts[r];
        displ[r] = 4 * sh.offsets[r];
    }
    const char *sc = getenv("ST_SIDE_CHANNEL");
    const bool side_on = !(sc && std::strcmp(sc, "0") == 0);
    Coll *bk = side_on ? co.side() : &co;
    // ST_SIDE_INLINE=1 (test hook): the RCCL issue order on a host transport -- the side channel's
    // calls from this thread at the same program points, the worker only for rank 0's ordering
    const bool inline_coll = !side_on || bk->enqueues() || getenv("ST_SIDE_INLINE");
    // the side context's stream carries the side channel's collectives and, on rank 0, the Morton
    // order and placement behind them (the context's side stream is the N-D fix-up's)
    st_ctx *mc = c;
    if (side_on) {
        if (!c->aux) ST_REQUIRE(st_ctx_create(c->device, &c->aux) == ST_OK, ST_ERR_HIP, "sog: side context");
        mc = c->aux;
    }
    const hipStream_t cs = mc->stream;
    float *gx = nullptr, *gy = nullptr, *gz = nullptr;
    uint32_t *pos = nullptr, *gath = nullptr;
    if (root) {
        gx = wsT<float>(c, "mg.gx", N);
        gy = wsT<float>(c, "mg.gy", N);
        gz = wsT<float>(c, "mg.gz", N);
        pos = wsT<uint32_t>(c, "mg.pos", N);
        gath = wsT<uint32_t>(c, "mg.gath", N * 5);
    }
    uint8_t *loc[6];
    for (int i = 0; i < ntex; ++i)  // (the scales / sh0 texels are rank 0's, in global row order)
        loc[i] = (i == 3 || i == 4) ? nullptr : wsT<uint8_t>(c, std::string("mg.loc.") + texn[i], sh.n * 4 + 4);
    uint8_t *dst[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (root) {
        uint8_t *o[6] = {out->means_l, out->means_u, out->quats, out->scales, out->sh0, out->shn_labels};
        for (int i = 0; i < 6; ++i) dst[i] = o[i];
    }
    Events ev;  // cols, xyz, tex, gath, side done, placed
    ST_HIP(hipEventRecord(ev[0], c->stream));  // the member columns are in place
    std::unique_ptr<SideWorker> wk;
    if (side_on) wk = std::make_unique<SideWorker>(c->device, &co, bk);
    auto on_side = [&](std::function<void()> f) {  // rank 0's ordering work
        if (wk) wk->push(std::move(f));
        else f();
    };
    auto side_coll = [&](std::function<void()> f) {  // the side channel's collectives
        if (inline_coll) f();
        else wk->push(std::move(f));
    };
    side_coll([&] {
        ST_HIP(hipStreamWaitEvent(cs, ev[0], 0));
        bk->gatherv(m[0], 4 * sh.n, gx, bytes, displ, 0, cs);
        bk->gatherv(m[1], 4 * sh.n, gy, bytes, displ, 0, cs);
        bk->gatherv(m[2], 4 * sh.n, gz, bytes, displ, 0, cs);
        ST_HIP(hipEventRecord(ev[1], cs));
    });
    if (root)
        on_side([&] {
            ST_HIP(hipStreamWaitEvent(mc->stream, ev[1], 0));
            auto *idx = wsT<uint32_t>(mc, "mg.idx", N);
            iota_u32(mc, idx, N);
            morton_order_dev(mc, gx, gy, gz, idx, N);
            hipLaunchKernelGGL(k_invert_u32, dim3(grid_for(N, 256, 8192)), dim3(256), 0, mc->stream, idx, N, pos);
            ST_LAUNCH_CHECK();
        });

    // global NaN-ignoring extents of x, y, z (write-sog.ts:161-187)
    double lo[3], hi[3];
    {
        minmax_dev(c, m, 3, sh.n, lo, hi);
        double h6[6] = {lo[0], lo[1], lo[2], -hi[0], -hi[1], -hi[2]};
        auto *d6 = wsT<double>(c, "mg.ext", 6);
        ST_HIP(hipMemcpyAsync(d6, h6, 48, hipMemcpyHostToDevice, c->stream));
        co.allreduce(d6, 6, Dt::F64, Op::Min, c->stream);
        ST_HIP(hipMemcpyAsync(h6, d6, 48, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        for (int a = 0; a < 3; ++a) {
            lo[a] = h6[a];
            hi[a] = -h6[3 + a];
        }
    }
    // cluster1d of the scales and of the colours (write-sog.ts:245-268) over the gathered global
    // columns, as on one device: not a sharded k-means -- 2 x 10 latency-bound iterations whose
    // all-reduces, read-backs and sequential hand-offs cost every rank more than moving the
    // columns (28 B per row).  The scales on rank 0, the colours on rank 1 from draw 0 (its
    // re-seed draws follow the scales': kept when the scales took none, rerun after them
    // otherwise); with one rank both on rank 0, the colours on a side context
    // (cluster1d_pair_dev).  The scales / sh0 texels go in global row order into the gather
    // buffer rank 0 places from; every rank takes the draws both consumed.
    uint64_t cursor = 0;
    auto *cb = wsT<float>(c, "mg.cb", 256);
    st_sog_meta lm{};
    {
        const int cr = co.world > 1 ? 1 : 0;  // the colours' rank
        const bool mine_c = co.rank == cr;
        float *gs = root ? wsT<float>(c, "mg.g1s", N * 3) : nullptr;    // scale_0..2
        float *gc = mine_c ? wsT<float>(c, "mg.g1c", N * 4) : nullptr;  // f_dc_0..2, opacity
        std::vector<Coll::Gather> g7;  // one group: rank 0's and rank 1's gathers move at once
        for (int i = 0; i < 3; ++i) g7.push_back({m[3 + i], 4 * sh.n, gs ? gs + N * i : nullptr, 0});
        for (int i = 0; i < 4; ++i) g7.push_back({m[6 + i], 4 * sh.n, gc ? gc + N * i : nullptr, cr});
        co.gatherv_many(g7, bytes, displ, c->stream);
        const float *sc3[3] = {gs, gs + N, gs + 2 * N};
        const float *co3[3] = {gc, gc + N, gc + 2 * N};
        auto *slab = root ? wsT<uint8_t>(c, "mg.slab", N * 3) : nullptr;
        auto *clab = mine_c ? wsT<uint8_t>(c, "mg.clab", N * 3) : nullptr;
        auto *cb_c = wsT<float>(c, "mg.cb_c", 256);
        auto *dused = wsT<unsigned long long>(c, "mg.used1d", 1);
        auto *hused = static_cast<unsigned long long *>(pinned_slot(c, "mg.used1d", 8));
        // rank `from`'s count of draws, on every rank
        auto share = [&](uint64_t v, int from) -> uint64_t {
            if (co.rank == from) {
                *hused = v;
                ST_HIP(hipMemcpyAsync(dused, hused, 8, hipMemcpyHostToDevice, c->stream));
            }
            co.broadcast(dused, 8, from, c->stream);
            ST_HIP(hipMemcpyAsync(hused, dused, 8, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipStreamSynchronize(c->stream));
            return *hused;
        };
        if (cr == 0) {
            if (!mc->aux) ST_REQUIRE(st_ctx_create(c->device, &mc->aux) == ST_OK, ST_ERR_HIP, "sog: side context");
            cursor += cluster1d_pair_dev(c, mc->aux, sc3, co3, N, iters, draws, ndraws, cb, slab, cb_c, clab);
        } else {
            uint64_t used_s = 0, used_c = 0;
            if (root) used_s = cluster1d_dev(c, sc3, 3, N, iters, draws, ndraws, cb, slab);
            if (mine_c) used_c = cluster1d_dev(c, co3, 3, N, iters, draws, ndraws, cb_c, clab);
            used_s = share(used_s, 0);
            if (mine_c && used_s)  // the scales took draws: the colours' k-means starts after them
                used_c = cluster1d_dev(c, co3, 3, N, iters, draws + used_s, ndraws - used_s, cb_c, clab);
            used_c = share(used_c, cr);
            cursor += used_s + used_c;
            // the colours' texels (global row order) and codebook to rank 0
            uint8_t *ctex = root ? (uint8_t *)(gath + N * 4) : mine_c ? wsT<uint8_t>(c, "mg.ctex", N * 4) : nullptr;
            if (mine_c) sog_table_rows(c, N, clab, gc + N * 3, ctex);
            co.sendrecv(ctex, 4 * N, cr, 0, c->stream);
            co.sendrecv(cb_c, 1024, cr, 0, c->stream);
        }
        if (root) {
            ST_HIP(hipMemcpyAsync(meta->scales_codebook, cb, 1024, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipMemcpyAsync(meta->sh0_codebook, cb_c, 1024, hipMemcpyDeviceToHost, c->stream));
            sog_table_rows(c, N, slab, nullptr, (uint8_t *)(gath + N * 3));
            if (cr == 0) sog_table_rows(c, N, clab, gc + N * 3, (uint8_t *)(gath + N * 4));
        }
    }

    // this rank's means / quats texels in local row order (4 bytes per row and texture)
    auto *rows = wsT<uint32_t>(c, "mg.iota", sh.n + 1);
    if (sh.n) iota_u32(c, rows, sh.n);
    st_sog_textures lt{loc[0], loc[1], loc[2], nullptr, nullptr, nullptr, nullptr};
    sog_scatter_dev(c, t, rows, lo, hi, nullptr, nullptr, nullptr, &lm, &lt);
    if (root) {
        for (int a = 0; a < 3; ++a) {
            meta->means_min[a] = lm.means_min[a];
            meta->means_max[a] = lm.means_max[a];
        }
    }
    ST_HIP(hipEventRecord(ev[2], c->stream));
    side_coll([&] {
        ST_HIP(hipStreamWaitEvent(cs, ev[2], 0));
        for (int i = 0; i < 3; ++i) bk->gatherv(loc[i], 4 * sh.n, gath ? gath + N * i : nullptr, bytes, displ, 0, cs);
        ST_HIP(hipEventRecord(ev[3], cs));
    });
    if (root)
        on_side([&] {
            ST_HIP(hipStreamWaitEvent(mc->stream, ev[3], 0));
            for (int i = 0; i < 5; ++i) {
                ST_HIP(hipMemsetAsync(dst[i], 0, texels * 4, mc->stream));
                hipLaunchKernelGGL(k_place, dim3(grid_for(N, 256, 8192)), dim3(256), 0, mc->stream, gath + N * i, pos,
                                   N, (uint32_t *)dst[i]);
                ST_LAUNCH_CHECK();
            }
            ST_HIP(hipEventRecord(ev[5], mc->stream));
        });

    if (root) meta->sh_bands = C == 15 ? 3 : C == 8 ? 2 : C == 3 ? 1 : 0;
    uint32_t *gath5 = nullptr;
    if (C) {
        const int D = 3 * C;
        auto *cen = wsT<float>(c, "mg.shcen", (size_t)pal * D);
        auto *labels = wsT<uint32_t>(c, "mg.shlab", sh.n + 1);
        Points P{&sh, false, D, 1, sh.n, N, {}};
        P.pts.assign(t->cols + 14, t->cols + 14 + D);
        cursor += kmeans_sharded(c, co, P, pal, iters, draws + cursor, ndraws - cursor, cen, labels, "mg.kn");
        // the codebook of the palette (identical input and draws on every rank)
        std::vector<const float *> ccols(D);
        for (int i = 0; i < D; ++i) ccols[i] = cen + (uint64_t)i * pal;
        auto *cl = wsT<uint8_t>(c, "mg.cl", (size_t)pal * D);
        cursor += cluster1d_dev(c, ccols.data(), D, (uint64_t)pal, iters, draws + cursor, ndraws - cursor, cb, cl);
        st_sog_textures lt2{};
        lt2.shn_labels = loc[5];
        sog_scatter_dev(c, t, rows, lo, hi, nullptr, nullptr, labels, &lm, &lt2);
        gath5 = root ? wsT<uint32_t>(c, "mg.gath5", N) : nullptr;
        co.gatherv(loc[5], 4 * sh.n, gath5, bytes, displ, 0, c->stream);
        if (root) {
            meta->palette_size = pal;
            meta->shn_width = cw;
            meta->shn_height = chh;
            ST_HIP(hipMemcpyAsync(meta->shn_codebook, cb, 1024, hipMemcpyDeviceToHost, c->stream));
            ST_HIP(hipMemsetAsync(out->shn_centroids, 0, (size_t)cw * chh * 4, c->stream));
            shn_centroids_dev(c, cl, C, pal, out->shn_centroids);
        }
    }
    if (wk) wk->drain();  // every side task has been issued (and, host-staged, has completed)
    if (side_on) {  // this stream continues after the side stream's gathers and rank 0's placement
        ST_HIP(hipEventRecord(ev[4], cs));
        ST_HIP(hipStreamWaitEvent(c->stream, ev[4], 0));
        if (root) ST_HIP(hipStreamWaitEvent(c->stream, ev[5], 0));
    }
    if (root && C) {  // pos is in place: on c->stream or behind ev[5]
        ST_HIP(hipMemsetAsync(dst[5], 0, texels * 4, c->stream));
        hipLaunchKernelGGL(k_place, dim3(grid_for(N, 256, 8192)), dim3(256), 0, c->stream, gath5, pos, N,
                           (uint32_t *)dst[5]);
        ST_LAUNCH_CHECK();
    }
    ST_HIP(hipStreamSynchronize(c->stream));
    return cursor;
}

// ST_COLL_TRACE=<dir> (diagnostics): every collective this rank issues, in the order its host
// threads issue them, one line per call appended to <dir>/coll_rank<r>.txt --
// "<channel> <op> <type/bytes> <root | from to>", the byte counts the ones every rank passes
// alike (a gatherv logs the total).  With RCCL (and ST_SIDE_INLINE=1 on a host transport) both
// channels are issued from the rank's main thread, so the files of all ranks must be identical:
// the issue-order argument of DESIGN.md (e) that a first RCCL run depends on.
struct TraceLog {
    std::mutex mu;
    FILE *f = nullptr;
    ~TraceLog() {
        if (f) fclose(f);
    }
    void put(int ch, const char *op, unsigned long long a, long long b = -1, long long c = -1) {
        std::lock_guard<std::mutex> lk(mu);
        if (!f) return;
        fprintf(f, "%d %s %llu", ch, op, a);
        if (b >= 0) fprintf(f, " %lld", b);
        if (c >= 0) fprintf(f, " %lld", c);
        fputc('\n', f);
        fflush(f);
    }
};
struct TraceColl : Coll {
    Coll *in;
    int ch;
    std::shared_ptr<TraceLog> log;
    std::unique_ptr<TraceColl> side_;
    TraceColl(Coll *inner, int channel, std::shared_ptr<TraceLog> l) : in(inner), ch(channel), log(std::move(l)) {
        rank = in->rank;
        world = in->world;
    }
    void allreduce(void *buf, size_t count, Dt dt, Op op, hipStream_t s) override {
        log->put(ch, op == Op::Sum ? (dt == Dt::F64 ? "allreduce_sum_f64" : "allreduce_sum_i32")
                                   : (dt == Dt::F64 ? "allreduce_min_f64" : "allreduce_min_i32"),
                 count);
        in->allreduce(buf, count, dt, op, s);
    }
    void broadcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        log->put(ch, "broadcast", bytes, root);
        in->broadcast(buf, bytes, root, s);
    }
    void allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        log->put(ch, "allgather", bytes);
        in->allgather(send, recv, bytes, s);
    }
    void gatherv(const void *send, size_t mybytes, void *recv, const std::vector<size_t> &bytes,
                 const std::vector<size_t> &displ, int root, hipStream_t s) override {
        unsigned long long tot = 0;
        for (size_t b : bytes) tot += b;
        log->put(ch, "gatherv", tot, root);
        in->gatherv(send, mybytes, recv, bytes, displ, root, s);
    }
    void gatherv_many(const std::vector<Gather> &gs, const std::vector<size_t> &bytes,
                      const std::vector<size_t> &displ, hipStream_t s) override {
        unsigned long long tot = 0;
        for (size_t b : bytes) tot += b;
        for (const Gather &g : gs) log->put(ch, "gatherv", tot, g.root);
        in->gatherv_many(gs, bytes, displ, s);
    }
    void sendrecv(void *buf, size_t bytes, int from, int to, hipStream_t s) override {
        log->put(ch, "sendrecv", bytes, from, to);
        in->sendrecv(buf, bytes, from, to, s);
    }
    void abort() override { in->abort(); }
    Coll *side() override {
        if (!side_) side_ = std::make_unique<TraceColl>(in->side(), ch + 1, log);
        return side_.get();
    }
    bool enqueues() const override { return in->enqueues(); }
};

// a failure on this rank aborts the job's channels: the peers' collectives fail instead of
// waiting for this rank (the communicator is not usable afterwards)
uint64_t sog_sharded(st_ctx *c, Coll &co, const st_table *const *tabs, int ntab, int iters, const double *draws,
                     uint64_t ndraws, st_sog_meta *meta, const st_sog_textures *out, uint64_t *n_global = nullptr) {
    std::unique_ptr<TraceColl> tc;
    if (const char *dir = getenv("ST_COLL_TRACE")) {
        auto log = std::make_shared<TraceLog>();
        const std::string path = std::string(dir) + "/coll_rank" + std::to_string(co.rank) + ".txt";
        log->f = fopen(path.c_str(), "a");
        ST_REQUIRE(log->f, ST_ERR_ARG, "ST_COLL_TRACE: cannot open " + path);
        tc = std::make_unique<TraceColl>(&co, 0, log);
    }
    Coll &cc = tc ? *tc : co;
    try {
        return sog_sharded_rank(c, cc, tabs, ntab, iters, draws, ndraws, meta, out, n_global);
    } catch (...) {
        co.abort();
        throw;
    }
}

}  // namespace st

// ---------------------------------------------------------------------------
// C-ABI
using namespace st;

struct st_comm {
    std::unique_ptr<Coll> coll;
};

// a process-local set of ranks: one (context, host thread) per rank
struct st_group {
    std::vector<st_ctx *> ctx;
    std::vector<int32_t> devices;
    bool host_staged = false;
    std::vector<std::unique_ptr<Coll>> coll;
    std::mutex run_mu;    // one group call at a time (the contexts and collectives are shared)
    std::string broken;  // non-empty: the collectives could not be rebuilt after a failure
    ~st_group() {
        coll.clear();
        for (auto *c : ctx) st_ctx_destroy(c);
    }
    // the collectives of every rank: RCCL communicators (ncclCommInitAll) or one host hub
    void make_colls() {
        const int n = (int)ctx.size();
        coll.clear();
        if (host_staged) {
            auto hub = std::make_shared<HostHub>(n);
            for (int r = 0; r < n; ++r) {
                auto hc = std::make_unique<HostColl>();
                hc->hub = hub;
                hc->rank = r;
                hc->world = n;
                coll.push_back(std::move(hc));
            }
        } else {
            std::vector<ncclComm_t> comms(n);
            ST_NCCL(ncclCommInitAll(comms.data(), n, devices.data()));
            for (int r = 0; r < n; ++r) {
                auto rc = std::make_unique<RcclColl>();
                rc->comm = comms[r];
                rc->rank = r;
                rc->world = n;
                coll.push_back(std::move(rc));
            }
        }
    }
    // f(rank) on every rank's thread; the first failure aborts the other ranks' collectives and
    // is rethrown once every thread has returned.  The aborted collectives are then rebuilt, so a
    // recoverable error (too few draws, an unsupported column) leaves the group usable.
    template <typename F>
    void run(F &&f) {
        std::lock_guard<std::mutex> lk(run_mu);
        if (!broken.empty()) throw Error(ST_ERR_INTERNAL, "multi-GPU group unusable: " + broken);
        const int n = (int)ctx.size();
        std::vector<std::exception_ptr> err(n);
        std::vector<std::thread> th;
        std::atomic<bool> failed{false};
        for (int r = 0; r < n; ++r)
            th.emplace_back([&, r] {
                try {
                    use_device(ctx[r]);
                    f(r);
                } catch (...) {
                    err[r] = std::current_exception();
                    if (!failed.exchange(true))
                        for (auto &cl : coll) cl->abort();
                }
            });
        for (auto &t : th) t.join();
        if (!failed.load()) return;
        // every rank thread has returned: drain the streams, then replace the collectives
        for (auto *c : ctx) {
            use_device(c);
            (void)hipStreamSynchronize(c->stream);
            (void)hipGetLastError();
        }
        try {
            make_colls();
        } catch (const std::exception &e) {
            broken = e.what();
        }
        // the first failure that is not the abort it caused in the other ranks
        std::exception_ptr first;
        for (auto &e : err) {
            if (!e) continue;
            try {
                std::rethrow_exception(e);
            } catch (const Error &x) {
                if (std::string(x.what()).find("another rank failed") == std::string::npos) {
                    first = e;
                    break;
                }
            } catch (...) {
                first = e;
                break;
            }
            if (!first) first = e;
        }
        std::rethrow_exception(first);
    }
};

namespace {
std::mutex g_group_mu;
std::shared_ptr<st_group> g_group;  // st_set_devices (a caller holds its own reference while it runs)
int g_ndev = 1;
std::atomic<bool> g_env_done{false};  // ST_NUM_GPUS applied (or overridden by st_set_devices)

template <typename F>
int guarded_m(F &&f) {
    try {
        f();
        return ST_OK;
    } catch (const st::Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return ST_ERR_INTERNAL;
    }
}

st_group *group_new(const int32_t *devices, int n, bool host_staged) {
    auto g = std::make_unique<st_group>();
    for (int r = 0; r < n; ++r) {
        st_ctx *c = nullptr;
        const int rc = st_ctx_create(devices[r], &c);
        if (rc != ST_OK) throw Error(rc, std::string("group: ") + st_last_error());
        g->ctx.push_back(c);
    }
    g->devices.assign(devices, devices + n);
    g->host_staged = host_staged;
    g->make_colls();
    return g.release();
}

// rows [lo, hi) of the concatenation of host tables (every column of each table, as given),
// uploaded into rank-local device columns: one device table per host table part
struct RankSlice {
    std::vector<std::vector<float *>> cols;
    std::vector<st_table> tabs;
    std::vector<const st_table *> ptrs;
};

RankSlice upload_slice(st_ctx *c, const st_table *const *tabs, int ntab, uint64_t lo, uint64_t hi) {
    RankSlice s;
    s.cols.resize(ntab);
    s.tabs.resize(ntab);
    uint64_t off = 0;
    std::vector<HostXfer> up;  // each rank's host thread stages its own slice (staged_h2d)
    for (int t = 0; t < ntab; ++t) {
        const uint64_t a = std::max(lo, off), b = std::min(hi, off + tabs[t]->n);
        const uint64_t m = b > a ? b - a : 0;
        for (int j = 0; j < tabs[t]->ncol; ++j) {
            float *d = wsT<float>(c, "gs.t" + std::to_string(t) + "." + std::to_string(j), m + 1);
            up.push_back(HostXfer{const_cast<float *>(tabs[t]->cols[j] + (a - off)), d, 4 * m});
            s.cols[t].push_back(d);
        }
        s.tabs[t] = *tabs[t];
        s.tabs[t].n = m;
        s.tabs[t].cols = s.cols[t].data();
        off += tabs[t]->n;
    }
    staged_h2d(c, up);
    for (auto &t : s.tabs) s.ptrs.push_back(&t);
    return s;
}
}  // namespace

// the group form of writeSog from host tables; textures on rank 0's device (dev_out) and,
// if host_out, copied there
static uint64_t group_sog(st_group *g, const st_table *const *tabs, int ntab, const uint64_t *splits, int iters,
                          const double *draws, uint64_t ndraws, st_sog_meta *meta, const st_sog_textures *dev_out,
                          const st_action *const *actions = nullptr, const int32_t *nactions = nullptr,
                          uint64_t *n_out = nullptr) {
    uint64_t N = 0;
    for (int t = 0; t < ntab; ++t) N += tabs[t]->n;
    const int world = (int)g->ctx.size();
    if (splits) {
        ST_REQUIRE(splits[0] == 0 && splits[world] == N, ST_ERR_ARG, "group: splits must run from 0 to the row count");
        for (int r = 0; r < world; ++r) ST_REQUIRE(splits[r] <= splits[r + 1], ST_ERR_ARG, "group: splits must ascend");
    }
    std::vector<uint64_t> used(world, 0);
    g->run([&](int r) {
        st_ctx *c = g->ctx[r];
        const uint64_t lo = splits ? splits[r] : N * r / world, hi = splits ? splits[r + 1] : N * (r + 1) / world;
        RankSlice s = upload_slice(c, tabs, ntab, lo, hi);
        // each input's processDataTable actions on this rank's part of it: every action is row-local
        // (transform) or order-preserving row selection (filters) or a renaming (filterBands against
        // the input's own band, the same on every rank), so the parts concatenate to the processed input
        std::vector<ProcessedF32> pr(actions ? ntab : 0);
        for (int t = 0; t < ntab && actions; ++t) {
            if (!nactions[t]) continue;
            chain_apply_f32(c, s.ptrs[t], actions[t], nactions[t], "gp" + std::to_string(t), pr[t]);
            s.ptrs[t] = &pr[t].t;
        }
        uint64_t nr = 0;
        used[r] = sog_sharded(c, *g->coll[r], s.ptrs.data(), ntab, iters, draws, ndraws, meta, dev_out, &nr);
        if (r == 0 && n_out) *n_out = nr;
    });
    for (int r = 1; r < world; ++r)
        ST_REQUIRE(used[r] == used[0], ST_ERR_INTERNAL, "multi-GPU: ranks consumed different draw counts");
    return used[0];
}

struct GroupTex {
    st_sog_textures t{};
};

static GroupTex group_tex(st_ctx *c, uint64_t N, int C) {
    int32_t W, H, pal, cw, chh;
    st_sog_geometry(N, C, &W, &H, &pal, &cw, &chh);
    const uint64_t tex = (uint64_t)W * H * 4;
    GroupTex g;
    g.t.means_l = wsT<uint8_t>(c, "gs.ml", tex);
    g.t.means_u = wsT<uint8_t>(c, "gs.mu", tex);
    g.t.quats = wsT<uint8_t>(c, "gs.q", tex);
    g.t.scales = wsT<uint8_t>(c, "gs.sc", tex);
    g.t.sh0 = wsT<uint8_t>(c, "gs.sh0", tex);
    if (C) {
        g.t.shn_labels = wsT<uint8_t>(c, "gs.shl", tex);
        g.t.shn_centroids = wsT<uint8_t>(c, "gs.shc", (uint64_t)cw * chh * 4);
    }
    return g;
}

// band of the combined tables (union of names, write-sog.ts:296)
static int union_coeffs(const st_table *const *tabs, int ntab) {
    int miss = -1;
    for (int i = 0; i < 45 && miss < 0; ++i) {
        char nm[32];
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        bool any = false;
        for (int t = 0; t < ntab; ++t) any = any || find_col(tabs[t], nm) >= 0;
        if (!any) miss = i;
    }
    return miss == 9 ? 3 : miss == 24 ? 8 : miss == -1 ? 15 : 0;
}

extern "C" {

int st_comm_unique_id(uint8_t id[128]) {
    return guarded_m([&] {
        ST_REQUIRE(id, ST_ERR_ARG, "NULL argument");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
        ncclUniqueId u;
        ST_NCCL(ncclGetUniqueId(&u));
        std::memcpy(id, &u, 128);
    });
}

int st_comm_init_rank(st_ctx *c, int32_t world, int32_t rank, const uint8_t id[128], st_comm **out) {
    return guarded_m([&] {
        ST_REQUIRE(c && id && out && world >= 1 && rank >= 0 && rank < world, ST_ERR_ARG, "bad argument");
        use_device(c);
        auto rc = std::make_unique<RcclColl>();
        ncclUniqueId u;
        std::memcpy(&u, id, 128);
        ST_NCCL(ncclCommInitRank(&rc->comm, world, u, rank));
        rc->rank = rank;
        rc->world = world;
        auto *cm = new st_comm();
        cm->coll = std::move(rc);
        *out = cm;
    });
}

int st_comm_init_host(st_ctx *c, int32_t world, int32_t rank, const char *name, uint64_t slot_bytes,
                      double timeout_s, st_comm **out) {
    return guarded_m([&] {
        ST_REQUIRE(c && name && out && world >= 1 && rank >= 0 && rank < world, ST_ERR_ARG, "bad argument");
        use_device(c);
        auto *cm = new st_comm();
        try {
            cm->coll = make_shm_coll(world, rank, name, slot_bytes ? (size_t)slot_bytes : (size_t)32 << 20, timeout_s);
        } catch (...) {
            delete cm;
            throw;
        }
        *out = cm;
    });
}

void st_comm_destroy(st_comm *cm) { delete cm; }

int st_comm_count(const st_comm *cm, int32_t *count) {
    return guarded_m([&] {
        ST_REQUIRE(cm && count, ST_ERR_ARG, "NULL argument");
        const auto *rc = dynamic_cast<const RcclColl *>(cm->coll.get());
        *count = rc ? rc->count() : cm->coll->world;
    });
}

int st_dev_sog_sharded(st_ctx *c, st_comm *cm, const st_table *const *locals, int32_t nlocal, int32_t iters,
                       const double *draws, uint64_t ndraws, uint64_t *used, st_sog_meta *meta,
                       const st_sog_textures *out) {
    return guarded_m([&] {
        ST_REQUIRE(c && cm && locals && nlocal >= 1 && draws, ST_ERR_ARG, "NULL argument");
        for (int i = 0; i < nlocal; ++i) ST_REQUIRE(locals[i], ST_ERR_ARG, "NULL table");
        if (cm->coll->rank == 0) ST_REQUIRE(meta && out, ST_ERR_ARG, "rank 0 needs meta and outputs");
        const uint64_t u = sog_sharded(c, *cm->coll, locals, nlocal, iters, draws, ndraws, meta, out);
        if (used) *used = u;
    });
}

int st_group_create(const int32_t *devices, int32_t n, int32_t host_staged, st_group **out) {
    return guarded_m([&] {
        ST_REQUIRE(devices && n >= 1 && out, ST_ERR_ARG, "bad argument");
        *out = group_new(devices, n, host_staged != 0);
    });
}

void st_group_destroy(st_group *g) { delete g; }

int st_group_sog(st_group *g, const st_table *const *tables, int32_t ntables, const uint64_t *splits, int32_t iters,
                 const double *draws, uint64_t ndraws, uint64_t *used, st_sog_meta *meta,
                 const st_sog_textures *out) {
    return guarded_m([&] {
        ST_REQUIRE(g && tables && ntables >= 1 && meta && out, ST_ERR_ARG, "NULL argument");
        uint64_t N = 0;
        for (int t = 0; t < ntables; ++t) N += tables[t]->n;
        const int C = union_coeffs(tables, ntables);
        GroupTex dt = group_tex(g->ctx[0], N, C);
        const uint64_t u = group_sog(g, tables, ntables, splits, iters, draws, ndraws, meta, &dt.t);
        st_ctx *c = g->ctx[0];
        use_device(c);
        const uint64_t tex = (uint64_t)meta->width * meta->height * 4;
        uint8_t *dst[6] = {out->means_l, out->means_u, out->quats, out->scales, out->sh0, out->shn_labels};
        uint8_t *src[6] = {dt.t.means_l, dt.t.means_u, dt.t.quats, dt.t.scales, dt.t.sh0, dt.t.shn_labels};
        std::vector<HostXfer> down;
        for (int i = 0; i < (C ? 6 : 5); ++i) {
            ST_REQUIRE(dst[i], ST_ERR_ARG, "sog: texture output is NULL");
            down.push_back(HostXfer{dst[i], src[i], tex});
        }
        if (C) {
            ST_REQUIRE(out->shn_centroids, ST_ERR_ARG, "sog: shN outputs are NULL");
            down.push_back(HostXfer{out->shn_centroids, dt.t.shn_centroids,
                                    (size_t)meta->shn_width * meta->shn_height * 4});
        }
        staged_d2h(c, down);
        if (used) *used = u;
    });
}

int st_group_sog_bundle(st_group *g, const st_table *const *tables, int32_t ntables, const uint64_t *splits,
                        int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used, uint16_t dos_time,
                        uint16_t dos_date, uint8_t **out, uint64_t *out_size) {
    return guarded_m([&] {
        ST_REQUIRE(g && tables && ntables >= 1 && out && out_size, ST_ERR_ARG, "NULL argument");
        uint64_t N = 0;
        for (int t = 0; t < ntables; ++t) N += tables[t]->n;
        GroupTex dt = group_tex(g->ctx[0], N, union_coeffs(tables, ntables));
        st_sog_meta meta{};
        const uint64_t u = group_sog(g, tables, ntables, splits, iters, draws, ndraws, &meta, &dt.t);
        st_ctx *c = g->ctx[0];
        use_device(c);
        const uint8_t *view;
        uint64_t nb;
        sog_bundle_dev(c, meta, N, dt.t, dos_time, dos_date, &view, &nb);
        uint8_t *buf = (uint8_t *)std::malloc(nb);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "sog bundle: host allocation failed");
        std::memcpy(buf, view, nb);
        *out = buf;
        *out_size = nb;
        if (used) *used = u;
    });
}

int st_group_sog_bundle_process(st_group *g, const st_table *const *tables, int32_t ntables, const uint64_t *splits,
                                const st_action *const *actions, const int32_t *nactions, int32_t iters,
                                const double *draws, uint64_t ndraws, uint64_t *used, uint16_t dos_time,
                                uint16_t dos_date, uint8_t **out, uint64_t *out_size) {
    return guarded_m([&] {
        ST_REQUIRE(g && tables && ntables >= 1 && out && out_size && actions && nactions, ST_ERR_ARG, "NULL argument");
        for (int t = 0; t < ntables; ++t) ST_REQUIRE(nactions[t] == 0 || actions[t], ST_ERR_ARG, "NULL action list");
        uint64_t N0 = 0;
        for (int t = 0; t < ntables; ++t) N0 += tables[t]->n;
        // textures for the unprocessed row count and band: filters only shrink the table and
        // filterBands only lowers the band, so these hold the processed table's
        GroupTex dt = group_tex(g->ctx[0], N0, 15);
        st_sog_meta meta{};
        uint64_t N = 0;
        const uint64_t u = group_sog(g, tables, ntables, splits, iters, draws, ndraws, &meta, &dt.t, actions, nactions,
                                     &N);
        st_ctx *c = g->ctx[0];
        use_device(c);
        const uint8_t *view;
        uint64_t nb;
        sog_bundle_dev(c, meta, N, dt.t, dos_time, dos_date, &view, &nb);
        uint8_t *buf = (uint8_t *)std::malloc(nb);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "sog bundle: host allocation failed");
        std::memcpy(buf, view, nb);
        *out = buf;
        *out_size = nb;
        if (used) *used = u;
    });
}

int st_set_devices(int32_t ngpu) {
    g_env_done.store(true);  // an explicit choice overrides ST_NUM_GPUS
    return guarded_m([&] {
        int avail = 0;
        ST_HIP(hipGetDeviceCount(&avail));
        ST_REQUIRE(ngpu >= 1 && ngpu <= avail, ST_ERR_ARG,
                   "st_set_devices: ngpu must be in [1, " + std::to_string(avail) + "]");
        std::shared_ptr<st_group> fresh;
        if (ngpu > 1) {
            std::vector<int32_t> devs(ngpu);
            for (int i = 0; i < ngpu; ++i) devs[i] = i;
            fresh.reset(group_new(devs.data(), ngpu, false));
        }
        std::lock_guard<std::mutex> lk(g_group_mu);
        g_group = std::move(fresh);  // the old group goes when its last running call returns
        g_ndev = ngpu;
    });
}

int st_get_devices(int32_t *ngpu) {
    if (!ngpu) return ST_ERR_ARG;
    if (int rc = st::apply_env_devices()) return rc;
    *ngpu = g_ndev;
    return ST_OK;
}

}  // extern "C"

namespace st {
// ST_NUM_GPUS=<n> (the host's device-count switch): st_set_devices(n) before the first
// writeSog of the process unless the host chose explicitly; a bad value fails that call
int apply_env_devices() {
    static std::mutex mu;
    static int rc = ST_OK;
    static std::string msg;
    std::lock_guard<std::mutex> lk(mu);
    if (!g_env_done.exchange(true)) {
        const char *e = getenv("ST_NUM_GPUS");
        if (e && *e) {
            char *end = nullptr;
            const long n = strtol(e, &end, 10);
            if (*end || n < 1 || n > 1024) {
                rc = ST_ERR_ARG;
                msg = std::string("ST_NUM_GPUS: not a device count: ") + e;
            } else if ((rc = st_set_devices((int32_t)n)) != ST_OK) {
                msg = std::string("ST_NUM_GPUS: ") + st_last_error();
            }
        }
        // test hook: the default group as n host-staged ranks on device 0, so that the one-call
        // writers' multi-GPU branches run on a one-GPU box
        const char *gr = getenv("ST_DEFAULT_GROUP_RANKS");
        if (rc == ST_OK && gr && atoi(gr) > 1) {
            rc = guarded_m([&] {
                const int n = std::min(atoi(gr), 16);
                std::vector<int32_t> devs(n, 0);
                std::shared_ptr<st_group> fresh(group_new(devs.data(), n, true));
                std::lock_guard<std::mutex> lk(g_group_mu);
                g_group = std::move(fresh);
                g_ndev = n;
            });
            if (rc != ST_OK) msg = std::string("ST_DEFAULT_GROUP_RANKS: ") + st_last_error();
        }
    }
    if (rc != ST_OK) set_last_error(msg);
    return rc;
}
// the process-wide group of st_set_devices (empty: one device); the caller's copy keeps it alive
std::shared_ptr<st_group> default_group() {
    std::lock_guard<std::mutex> lk(g_group_mu);
    return g_group;
}
}  // namespace st
