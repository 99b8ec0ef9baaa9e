// st_shm.cpp -- the collectives of the sharded writeSog between PROCESSES through one POSIX
// shared-memory segment (st_coll.h make_shm_coll, C-ABI st_comm_init_host).
//
// What it is for: RCCL refuses two ranks on one GPU, so without it the one-process-per-GPU job
// (bench.py --gpus N, st_comm_* + st_dev_sog_sharded) could only be exercised on a node with N
// GPUs.  With it the same processes, the same library calls and the same two channels (the
// k-means all-reduces on the main one, the texel gathers on the side one, from another host
// thread) run as N processes on one card; only the bytes travel through host memory instead of
// xGMI.  It is a correctness transport, not a fast one (every rank reduces every slot).
//
// Layout: a header (barrier state of the two channels, the ranks' pids, an abort flag), then
// 2 x world staging slots of slot_bytes (pinned with hipHostRegister when the runtime allows, so
// the device copies into and out of them are DMA).  Each exchange moves at most one slot per rank
// per round: put (device -> own slot), barrier, read peers' slots (-> device or a host
// reduction), barrier.  Waits spin briefly, then yield, then sleep; they give up when another
// rank aborted, when a peer process has exited, or after timeout_s, and the failure aborts every
// rank of the job (they throw "multi-GPU: another rank failed").
#include <fcntl.h>
#include <signal.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <new>
#include <string>

#include "st_coll.h"
#include "st_internal.h"

namespace st {
namespace {

constexpr uint64_t kMagic = 0x31304d48535f5453ull;  // "ST_SHM01"
constexpr int kMaxRanks = 256;
constexpr double kAttachLimitS = 120;  // longest wait for every rank to attach
constexpr int kChannels = 2;

struct alignas(64) Chan {
    std::atomic<uint32_t> arrived;
    alignas(64) std::atomic<uint64_t> gen;
};

struct Header {
    std::atomic<uint64_t> magic;
    uint32_t world;
    uint32_t pad;
    uint64_t slot_bytes;
    std::atomic<uint32_t> attached;
    std::atomic<uint32_t> aborted;  // 0, or 1 + the rank that aborted
    std::atomic<int32_t> pid[kMaxRanks];
    Chan chan[kChannels];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free && std::atomic<uint32_t>::is_always_lock_free,
              "process-shared atomics must be lock-free");

size_t header_bytes() { return (sizeof(Header) + 4095) & ~size_t(4095); }

[[noreturn]] void sys_fail(const std::string &what) {
    throw Error(ST_ERR_INTERNAL, "shared-memory transport: " + what + ": " + std::strerror(errno));
}

// one mapping of the job's segment, shared by the main and side channel objects of a rank
struct Seg {
    std::string name;
    void *base = nullptr;
    size_t size = 0;
    Header *h = nullptr;
    char *slots = nullptr;
    size_t slot = 0;
    int world = 1, rank = 0;
    double timeout_s = 600;
    bool registered = false, unlinked = false;
    ~Seg() {
        if (registered) (void)hipHostUnregister(slots);
        if (base) munmap(base, size);
        if (rank == 0 && !unlinked && !name.empty()) shm_unlink(name.c_str());
    }
    char *slot_of(int ch, int r) const { return slots + ((size_t)ch * world + r) * slot; }
    void abort_job() {
        uint32_t z = 0;
        h->aborted.compare_exchange_strong(z, 1u + (uint32_t)rank);
    }
    // the first peer (pid set) whose process no longer exists, or -1
    int dead_peer() const {
        for (int r = 0; r < world; ++r) {
            const int32_t p = h->pid[r].load(std::memory_order_acquire);
            if (r != rank && p > 0 && kill(p, 0) != 0 && errno == ESRCH) return r;
        }
        return -1;
    }
    // spin, then yield, then sleep until done(); abort / dead peer / timeout throw
    template <typename F>
    void wait(F &&done, const char *what, double limit_s = 0) {
        if (limit_s <= 0) limit_s = timeout_s;
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        auto checked = t0;
        for (uint64_t i = 0;; ++i) {
            if (done()) return;
            if (h->aborted.load(std::memory_order_acquire))
                throw Error(ST_ERR_INTERNAL, "multi-GPU: another rank failed");
            if (i < 4096) {
                __builtin_ia32_pause();
                continue;
            }
            const auto now = clk::now();
            if (now - checked > std::chrono::milliseconds(100)) {
                checked = now;
                const int d = dead_peer();
                if (d >= 0) {
                    abort_job();
                    throw Error(ST_ERR_INTERNAL, "shared-memory transport: rank " + std::to_string(d) +
                                                     " exited during " + what);
                }
                if (std::chrono::duration<double>(now - t0).count() > limit_s) {
                    abort_job();
                    throw Error(ST_ERR_INTERNAL, std::string("shared-memory transport: no progress for ") +
                                                     std::to_string((int)limit_s) + " s during " + what);
                }
            }
            if (i < 8192) {
                sched_yield();
            } else {
                const timespec ts{0, 50 * 1000};
                nanosleep(&ts, nullptr);
            }
        }
    }
    void barrier(int ch, const char *what) {
        Chan &c = h->chan[ch];
        const uint64_t g = c.gen.load(std::memory_order_acquire);
        if (h->aborted.load(std::memory_order_acquire)) throw Error(ST_ERR_INTERNAL, "multi-GPU: another rank failed");
        if (c.arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)world) {
            c.arrived.store(0, std::memory_order_relaxed);
            c.gen.fetch_add(1, std::memory_order_release);
            return;
        }
        wait([&] { return c.gen.load(std::memory_order_acquire) != g; }, what);
    }
};

struct ShmColl : Coll {
    std::shared_ptr<Seg> seg;
    int ch = 0;
    std::unique_ptr<ShmColl> side_;
    std::vector<char> acc;
    ShmColl(std::shared_ptr<Seg> s, int channel) : seg(std::move(s)), ch(channel) {
        rank = seg->rank;
        world = seg->world;
    }
    bool enqueues() const override { return false; }
    Coll *side() override {
        ST_REQUIRE(ch == 0, ST_ERR_INTERNAL, "shared-memory transport: the side channel has no side channel");
        if (!side_) side_ = std::make_unique<ShmColl>(seg, 1);
        return side_.get();
    }
    void abort() override { seg->abort_job(); }
    char *mine() const { return seg->slot_of(ch, rank); }
    char *of(int r) const { return seg->slot_of(ch, r); }
    void put(const void *dev, size_t bytes, hipStream_t s) {
        if (bytes) {
            ST_HIP(hipMemcpyAsync(mine(), dev, bytes, hipMemcpyDeviceToHost, s));
            ST_HIP(hipStreamSynchronize(s));
        }
    }
    void get(void *dev, int r, size_t bytes, hipStream_t s) {
        if (bytes) ST_HIP(hipMemcpyAsync(dev, of(r), bytes, hipMemcpyHostToDevice, s));
    }
    size_t rounds(size_t bytes) const { return (bytes + seg->slot - 1) / seg->slot; }

    void allreduce(void *buf, size_t count, Dt dt, Op op, hipStream_t s) override {
        if (world == 1 || !count) return;
        const size_t es = dt == Dt::F64 ? 8 : 4, per = seg->slot / es;
        for (size_t a = 0; a < count; a += per) {
            const size_t m = std::min(per, count - a);
            char *b = static_cast<char *>(buf) + a * es;
            put(b, m * es, s);
            seg->barrier(ch, "allreduce");
            acc.assign(of(0), of(0) + m * es);
            for (int r = 1; r < world; ++r) {
                const char *src = of(r);
                if (dt == Dt::F64) {
                    for (size_t i = 0; i < m; ++i) {
                        double x, y;
                        std::memcpy(&x, acc.data() + 8 * i, 8);
                        std::memcpy(&y, src + 8 * i, 8);
                        x = op == Op::Sum ? x + y : std::min(x, y);
                        std::memcpy(acc.data() + 8 * i, &x, 8);
                    }
                } else {
                    for (size_t i = 0; i < m; ++i) {
                        int32_t x, y;
                        std::memcpy(&x, acc.data() + 4 * i, 4);
                        std::memcpy(&y, src + 4 * i, 4);
                        x = op == Op::Sum ? (int32_t)((uint32_t)x + (uint32_t)y) : std::min(x, y);
                        std::memcpy(acc.data() + 4 * i, &x, 4);
                    }
                }
            }
            seg->barrier(ch, "allreduce");  // every rank has read every slot
            ST_HIP(hipMemcpyAsync(b, acc.data(), m * es, hipMemcpyHostToDevice, s));
            ST_HIP(hipStreamSynchronize(s));
        }
    }
    void broadcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        if (world == 1 || !bytes) return;
        const size_t S = seg->slot;
        for (size_t a = 0; a < bytes; a += S) {
            const size_t m = std::min(S, bytes - a);
            char *b = static_cast<char *>(buf) + a;
            if (rank == root) put(b, m, s);
            seg->barrier(ch, "broadcast");
            if (rank != root) {
                get(b, root, m, s);
                ST_HIP(hipStreamSynchronize(s));
            }
            seg->barrier(ch, "broadcast");
        }
    }
    void allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        if (!bytes) return;
        if (world == 1) {
            if (recv != send) ST_HIP(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
            return;
        }
        const size_t S = seg->slot;
        for (size_t a = 0; a < bytes; a += S) {
            const size_t m = std::min(S, bytes - a);
            put(static_cast<const char *>(send) + a, m, s);
            seg->barrier(ch, "allgather");
            for (int r = 0; r < world; ++r) get(static_cast<char *>(recv) + bytes * r + a, r, m, s);
            ST_HIP(hipStreamSynchronize(s));
            seg->barrier(ch, "allgather");
        }
    }
    void gatherv(const void *send, size_t mybytes, void *recv, const std::vector<size_t> &bytes,
                 const std::vector<size_t> &displ, int root, hipStream_t s) override {
        if (world == 1) {
            if (mybytes) ST_HIP(hipMemcpyAsync(static_cast<char *>(recv) + displ[0], send, mybytes,
                                               hipMemcpyDeviceToDevice, s));
            return;
        }
        size_t mx = 0;
        for (size_t b : bytes) mx = std::max(mx, b);
        const size_t S = seg->slot;
        for (size_t a = 0; a < mx; a += S) {
            if (a < mybytes) put(static_cast<const char *>(send) + a, std::min(S, mybytes - a), s);
            seg->barrier(ch, "gatherv");
            if (rank == root) {
                for (int r = 0; r < world; ++r)
                    if (a < bytes[r]) get(static_cast<char *>(recv) + displ[r] + a, r, std::min(S, bytes[r] - a), s);
                ST_HIP(hipStreamSynchronize(s));
            }
            seg->barrier(ch, "gatherv");
        }
    }
    void sendrecv(void *buf, size_t bytes, int from, int to, hipStream_t s) override {
        if (world == 1 || from == to || !bytes) return;
        const size_t S = seg->slot;
        for (size_t a = 0; a < bytes; a += S) {
            const size_t m = std::min(S, bytes - a);
            char *b = static_cast<char *>(buf) + a;
            if (rank == from) put(b, m, s);
            seg->barrier(ch, "sendrecv");
            if (rank == to) {
                get(b, from, m, s);
                ST_HIP(hipStreamSynchronize(s));
            }
            seg->barrier(ch, "sendrecv");
        }
    }
};

void sleep_ms(int ms) {
    const timespec ts{0, ms * 1000000L};
    nanosleep(&ts, nullptr);
}

}  // namespace

std::unique_ptr<Coll> make_shm_coll(int world, int rank, const char *name, size_t slot_bytes, double timeout_s) {
    ST_REQUIRE(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world, ST_ERR_ARG,
               "shared-memory transport: world must be in [1, 256] and 0 <= rank < world");
    ST_REQUIRE(name && *name && std::strlen(name) <= 200, ST_ERR_ARG, "shared-memory transport: bad job name");
    for (const char *p = name; *p; ++p)
        ST_REQUIRE(std::isalnum((unsigned char)*p) || *p == '_' || *p == '-' || *p == '.', ST_ERR_ARG,
                   "shared-memory transport: the job name may hold [A-Za-z0-9_.-] only");
    ST_REQUIRE(slot_bytes >= 4096 && slot_bytes % 4096 == 0, ST_ERR_ARG,
               "shared-memory transport: slot_bytes must be a positive multiple of 4096");
    auto seg = std::make_shared<Seg>();
    seg->name = std::string("/st_") + name;
    seg->slot = slot_bytes;
    seg->world = world;
    seg->rank = rank;
    seg->timeout_s = timeout_s > 0 ? timeout_s : 600;
    seg->size = header_bytes() + (size_t)kChannels * world * slot_bytes;
    // the ranks meet within kAttachLimitS by default: a rank that died before attaching ends rank
    // 0's wait, and rank 0 unlinks the name, well before a launcher's first-stall kill (bench.py:
    // 600 s) could stop rank 0 with no destructor run and leave the segment in tmpfs.  A job that
    // sets its timeout explicitly (timeout_s > 0) waits that long instead -- ranks that start far
    // apart on purpose -- and ST_SHM_ATTACH_S overrides both
    double attach_s = timeout_s > 0 ? timeout_s : std::min(seg->timeout_s, kAttachLimitS);
    if (const char *e = getenv("ST_SHM_ATTACH_S"))
        if (atof(e) > 0) attach_s = atof(e);
    using clk = std::chrono::steady_clock;
    const auto deadline = clk::now() + std::chrono::duration<double>(attach_s);
    if (rank == 0) {
        const int fd = shm_open(seg->name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) {
            seg->name.clear();  // not ours: never unlink it
            sys_fail("shm_open(create) of a fresh job name");
        }
        if (ftruncate(fd, (off_t)seg->size) != 0) {
            close(fd);
            sys_fail("ftruncate");
        }
        seg->base = mmap(nullptr, seg->size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (seg->base == MAP_FAILED) {
            seg->base = nullptr;
            sys_fail("mmap");
        }
        seg->h = new (seg->base) Header();
        seg->h->world = (uint32_t)world;
        seg->h->slot_bytes = slot_bytes;
        for (auto &p : seg->h->pid) p.store(0, std::memory_order_relaxed);
        seg->h->magic.store(kMagic, std::memory_order_release);
    } else {
        for (;;) {
            const int fd = shm_open(seg->name.c_str(), O_RDWR, 0);
            if (fd >= 0) {
                struct stat st {};
                if (fstat(fd, &st) == 0 && (size_t)st.st_size >= seg->size) {
                    seg->base = mmap(nullptr, seg->size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                    close(fd);
                    if (seg->base == MAP_FAILED) {
                        seg->base = nullptr;
                        sys_fail("mmap");
                    }
                    break;
                }
                close(fd);
            } else if (errno != ENOENT) {
                sys_fail("shm_open(attach)");
            }
            ST_REQUIRE(clk::now() < deadline, ST_ERR_INTERNAL,
                       "shared-memory transport: rank 0 did not create the job's segment in time");
            sleep_ms(2);
        }
        seg->h = static_cast<Header *>(seg->base);
        while (seg->h->magic.load(std::memory_order_acquire) != kMagic) {
            ST_REQUIRE(clk::now() < deadline, ST_ERR_INTERNAL, "shared-memory transport: segment never initialised");
            sleep_ms(1);
        }
        ST_REQUIRE(seg->h->world == (uint32_t)world && seg->h->slot_bytes == slot_bytes, ST_ERR_ARG,
                   "shared-memory transport: the ranks disagree on world size or slot size");
    }
    seg->slots = static_cast<char *>(seg->base) + header_bytes();
    seg->h->pid[rank].store((int32_t)getpid(), std::memory_order_release);
    seg->h->attached.fetch_add(1, std::memory_order_acq_rel);
    seg->wait([&] { return seg->h->attached.load(std::memory_order_acquire) == (uint32_t)world; }, "attach",
              attach_s);
    if (rank == 0) {  // every rank has it mapped: the name can go
        shm_unlink(seg->name.c_str());
        seg->unlinked = true;
    }
    // pinned staging: the device copies in and out of the slots are then DMA (best effort)
    if (hipHostRegister(seg->slots, seg->size - header_bytes(), hipHostRegisterDefault) == hipSuccess)
        seg->registered = true;
    else
        (void)hipGetLastError();
    return std::make_unique<ShmColl>(seg, 0);
}

}  // namespace st
