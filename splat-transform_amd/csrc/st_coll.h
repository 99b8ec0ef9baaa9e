// st_coll.h -- the collectives one rank of the sharded writeSog uses (st_multi.hip), over three
// transports: RCCL (st_multi.hip: one process per GPU, or one process driving several GPUs),
// host hubs between the threads of one process (st_multi.hip), and a POSIX shared-memory hub
// between processes (st_shm.cpp: several one-rank processes on one GPU, where RCCL refuses two
// ranks on one device -- the same process layout as the 8-GPU job, rehearsed on one card).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <vector>

namespace st {

enum class Dt { F64, I32 };
enum class Op { Sum, Min };

// every call is stream-ordered on `s`
struct Coll {
    int rank = 0, world = 1;
    virtual ~Coll() = default;
    virtual void allreduce(void *buf, size_t count, Dt dt, Op op, hipStream_t s) = 0;
    virtual void broadcast(void *buf, size_t bytes, int root, hipStream_t s) = 0;
    // recv (every rank) = the ranks' `bytes`-sized sends, rank order
    virtual void allgather(const void *send, void *recv, size_t bytes, hipStream_t s) = 0;
    // root: recv[r] (at offset displ[r]) = rank r's send of bytes[r]; recv ignored elsewhere
    virtual void gatherv(const void *send, size_t mybytes, void *recv, const std::vector<size_t> &bytes,
                         const std::vector<size_t> &displ, int root, hipStream_t s) = 0;
    // several gathervs over the same shard layout, each to its own root (recv ignored off the
    // root): RCCL issues them as one group, so gathers into different roots move at once
    struct Gather {
        const void *send;
        size_t mybytes;
        void *recv;
        int root;
    };
    virtual void gatherv_many(const std::vector<Gather> &gs, const std::vector<size_t> &bytes,
                              const std::vector<size_t> &displ, hipStream_t s) {
        for (const Gather &g : gs) gatherv(g.send, g.mybytes, g.recv, bytes, displ, g.root, s);
    }
    // rank `to` receives rank `from`'s buf (every rank makes the call; the others pass through)
    virtual void sendrecv(void *buf, size_t bytes, int from, int to, hipStream_t s) = 0;
    // after abort() every call of every rank on this channel (and its side channel) throws
    virtual void abort() {}
    // a second channel over the same ranks, whose calls may run beside this one's (from another
    // host thread, on another stream): the bulk texel traffic of the writer.  Collective: every
    // rank asks for it at the same point; made once and kept.
    virtual Coll *side() = 0;
    // true: a call only enqueues device work on `s` and returns (RCCL).  The two channels' calls
    // are then issued from ONE host thread in program order, identical on every rank, so that
    // blocking collective kernels of the two channels can never wait on each other in opposite
    // orders on two ranks (two streams may share a hardware queue).  false: a call returns when
    // its data has moved (host-staged transports); the side channel's calls run on a worker
    // thread, the channels' hubs are independent.
    virtual bool enqueues() const = 0;
};

// the shared-memory transport of one process's rank (st_shm.cpp).  `name` identifies the job
// (every rank passes the same; [A-Za-z0-9_.-], at most 200 characters); rank 0 creates the
// segment /dev/shm/st_<name>, the others attach, and the name is unlinked as soon as every rank
// has attached (nothing stays in /dev/shm, whatever happens later).  slot_bytes: the staging
// slot of one rank on one channel (transfers larger than it move in several rounds).
// timeout_s: the longest a rank waits for its peers in one exchange before the job is aborted;
// a peer process that exits makes every waiting rank fail at once.
std::unique_ptr<Coll> make_shm_coll(int world, int rank, const char *name, size_t slot_bytes, double timeout_s);

}  // namespace st
