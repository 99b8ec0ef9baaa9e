// st_rccl.h -- the RCCL the library's collectives run on, loaded at run time (dlopen) instead of
// bound at link time.
//
// Linked with -lrccl, the library's NEEDED librccl.so.1 bound to whichever copy of that soname
// the process had loaded first: torch's bundled RCCL (2.26.6) under the Python host, the ROCm
// install's (/opt/rocm/lib, 2.27.7, the headers this file compiles against) under the Node host.
// One product ran on two RCCLs and reported neither.  Now both hosts open the same file by path,
// under a handle of its own (RTLD_LOCAL: torch.distributed keeps its copy, the library never
// resolves a symbol against it):
//   ST_RCCL unset      /opt/rocm/lib/librccl.so.1 (the ROCm install's RCCL)
//   ST_RCCL=<path>     that file
//   ST_RCCL=process    the copy of soname librccl.so.1 already in the process, if any (torch's
//                      under Python), else the loader's search path -- the pre-round-6 binding
// st_rccl_info (st_abi.h) reports the version (ncclGetVersion) and the file's real path; the
// bench line carries them (rccl_version, rccl_path).
#pragma once

#include <rccl/rccl.h>

#include <string>

namespace st {

struct RcclApi {
    decltype(&::ncclGetVersion) GetVersion;
    decltype(&::ncclGetErrorString) GetErrorString;
    decltype(&::ncclGetUniqueId) GetUniqueId;
    decltype(&::ncclCommInitRank) CommInitRank;
    decltype(&::ncclCommInitAll) CommInitAll;
    decltype(&::ncclCommSplit) CommSplit;
    decltype(&::ncclCommDestroy) CommDestroy;
    decltype(&::ncclCommAbort) CommAbort;
    decltype(&::ncclCommCount) CommCount;
    decltype(&::ncclAllReduce) AllReduce;
    decltype(&::ncclBroadcast) Broadcast;
    decltype(&::ncclAllGather) AllGather;
    decltype(&::ncclSend) Send;
    decltype(&::ncclRecv) Recv;
    decltype(&::ncclGroupStart) GroupStart;
    decltype(&::ncclGroupEnd) GroupEnd;
    int version = 0;   // ncclGetVersion
    std::string path;  // the loaded file (realpath)
    std::string how;   // "path" or "process"
};

// loads RCCL on first use (thread-safe); throws st::Error(ST_ERR_INTERNAL) if it cannot
const RcclApi &rccl();

}  // namespace st
