// st_rccl.cpp -- run-time binding of RCCL (see st_rccl.h for why and which file)
#include "st_rccl.h"

#include <dlfcn.h>
#include <limits.h>
#include <stdlib.h>

#include <cstring>
#include <mutex>

#include "st_internal.h"

namespace st {

namespace {

const char *kDefaultRccl = "/opt/rocm/lib/librccl.so.1";

template <typename T>
void sym(void *h, const char *name, T &out, const std::string &file) {
    dlerror();
    void *p = dlsym(h, name);
    ST_REQUIRE(p, ST_ERR_INTERNAL, std::string("RCCL: ") + file + " has no symbol " + name);
    out = reinterpret_cast<T>(p);
}

RcclApi load() {
    const char *env = getenv("ST_RCCL");
    RcclApi a;
    void *h = nullptr;
    std::string want;
    if (env && std::strcmp(env, "process") == 0) {
        // by soname: the copy already mapped (torch's under Python) if there is one
        a.how = "process";
        want = "librccl.so.1";
        h = dlopen(want.c_str(), RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen(want.c_str(), RTLD_NOW | RTLD_LOCAL);
    } else {
        // by path, its own handle: a file name with a '/' is matched against the loaded objects by
        // file identity, not by soname, so torch's librccl.so.1 is not reused for it
        a.how = "path";
        want = (env && *env) ? env : kDefaultRccl;
        h = dlopen(want.c_str(), RTLD_NOW | RTLD_LOCAL);
    }
    if (!h) {
        const char *why = dlerror();
        throw Error(ST_ERR_INTERNAL, "RCCL: cannot load " + want + ": " + (why ? why : "?") +
                                         " (set ST_RCCL to an RCCL library path, or to 'process')");
    }
    sym(h, "ncclGetVersion", a.GetVersion, want);
    sym(h, "ncclGetErrorString", a.GetErrorString, want);
    sym(h, "ncclGetUniqueId", a.GetUniqueId, want);
    sym(h, "ncclCommInitRank", a.CommInitRank, want);
    sym(h, "ncclCommInitAll", a.CommInitAll, want);
    sym(h, "ncclCommSplit", a.CommSplit, want);
    sym(h, "ncclCommDestroy", a.CommDestroy, want);
    sym(h, "ncclCommAbort", a.CommAbort, want);
    sym(h, "ncclCommCount", a.CommCount, want);
    sym(h, "ncclAllReduce", a.AllReduce, want);
    sym(h, "ncclBroadcast", a.Broadcast, want);
    sym(h, "ncclAllGather", a.AllGather, want);
    sym(h, "ncclSend", a.Send, want);
    sym(h, "ncclRecv", a.Recv, want);
    sym(h, "ncclGroupStart", a.GroupStart, want);
    sym(h, "ncclGroupEnd", a.GroupEnd, want);
    ST_REQUIRE(a.GetVersion(&a.version) == ncclSuccess, ST_ERR_INTERNAL, "RCCL: ncclGetVersion failed");
    Dl_info info;
    std::memset(&info, 0, sizeof info);
    a.path = want;
    if (dladdr(reinterpret_cast<void *>(a.GetVersion), &info) && info.dli_fname) {
        char real[PATH_MAX];
        a.path = realpath(info.dli_fname, real) ? real : info.dli_fname;
    }
    return a;  // the handle stays open for the life of the process
}

}  // namespace

const RcclApi &rccl() {
    static std::once_flag once;
    static RcclApi api;
    static std::string err;
    static int code = ST_OK;
    std::call_once(once, [] {
        try {
            api = load();
        } catch (const Error &e) {
            err = e.what();
            code = e.code;
        }
    });
    if (code != ST_OK) throw Error(code, err);
    return api;
}

}  // namespace st

extern "C" int st_rccl_info(int32_t *version, char *path, uint64_t path_len) {
    return st::guard([&] {
        const st::RcclApi &a = st::rccl();
        if (version) *version = a.version;
        if (path && path_len) {
            std::strncpy(path, a.path.c_str(), path_len - 1);
            path[path_len - 1] = 0;
        }
    });
}
