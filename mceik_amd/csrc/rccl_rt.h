// rccl_rt.h -- RCCL opened on first use (dlopen "librccl.so.1", the library
// torch's nccl backend loads), shared by the sampler's checkpoint gather
// (comm.hip) and the halo exchange of the block-decomposed solve across ranks
// (capi.hip).  The product library carries no link dependency on RCCL, and
// single-GPU callers never load it.  Not a public header.
#pragma once
#include <dlfcn.h>
#include <stdio.h>

#include <type_traits>

#include <rccl/rccl.h>

struct MceikRccl {
    bool ok = false;
    const char *(*GetErrorString)(ncclResult_t);
    ncclResult_t (*GetUniqueId)(ncclUniqueId *);
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
};

inline const MceikRccl &mceik_rccl()
{
    static MceikRccl r = [] {
        MceikRccl x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            fprintf(stderr, "mceik_hip: cannot load RCCL (%s)\n", dlerror());
            return x;
        }
        bool all = true;
        auto get = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) { fprintf(stderr, "mceik_hip: RCCL lacks %s\n", name); all = false; }
        };
        get(x.GetErrorString, "ncclGetErrorString");
        get(x.GetUniqueId, "ncclGetUniqueId");
        get(x.CommInitRank, "ncclCommInitRank");
        get(x.CommDestroy, "ncclCommDestroy");
        get(x.AllGather, "ncclAllGather");
        get(x.AllReduce, "ncclAllReduce");
        get(x.Send, "ncclSend");
        get(x.Recv, "ncclRecv");
        get(x.GroupStart, "ncclGroupStart");
        get(x.GroupEnd, "ncclGroupEnd");
        x.ok = all;
        return x;
    }();
    return r;
}
