// comm.hip -- multi-rank runs from C (include/mceik.h mceik_comm_*,
// mceik_mcmc_gather): the sampler's only collective, the checkpoint gather of
// every rank's chain shard to a root rank over RCCL (xGMI on one node;
// SURVEY s.8e).
//
// The reference's multi-rank flow is MPI end to end: broadcast.c:14-143 sends
// the catalogue/stations from the master, mpiutils.f90:346-426 splits the
// communicators, homog.c:343-415 has rank 0 gather and write.  Here a C/MPI
// main keeps MPI for launch and bootstrap only (one rank per GPU): rank 0
// makes the RCCL id, the main broadcasts its 128 bytes (MPI_Bcast), every
// rank builds the communicator and calls mceik_mcmc_gather at a checkpoint.
//
// RCCL is opened on first use (dlopen "librccl.so.1", the same library torch's
// nccl backend loads), so the product library carries no link dependency on
// it and single-GPU callers never load it.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/mceik.h"
#include "rccl_rt.h"
#include "mcmc_common.h"

// Runs the calling scope on `dev` and restores the caller's device.
struct DevScope {
    int prev = -1;
    explicit DevScope(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) hipSetDevice(dev);
        else prev = -1;
    }
    ~DevScope()
    {
        if (prev >= 0) hipSetDevice(prev);
    }
};

// true if p is device memory of GPU `dev` (the gather then receives into it)
static bool on_device(const void *p, int dev)
{
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice && a.device == dev;
}

struct mceik_comm {
    ncclComm_t comm;
    int nranks, rank, device;
    int *d_shard;          // [nranks][3] (chain_offset, nchains, local status) exchange buffer
    hipStream_t stream;    // the gather's own stream (non-blocking)
};

#define RCCLCHK(x)                                                                         \
    do {                                                                                   \
        ncclResult_t r_ = (x);                                                             \
        if (r_ != ncclSuccess) {                                                           \
            fprintf(stderr, "mceik_comm: %s failed: %s\n", #x, mceik_rccl().GetErrorString(r_)); \
            return -1;                                                                     \
        }                                                                                  \
    } while (0)
#define HIPCHK2(x)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "mceik_comm: %s failed: %s\n", #x, hipGetErrorString(e_));     \
            return -1;                                                                     \
        }                                                                                  \
    } while (0)

extern "C" int mceik_comm_available(void)
{
    return mceik_rccl().ok ? 1 : 0;
}

extern "C" int mceik_comm_unique_id(unsigned char id[MCEIK_COMM_ID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) == MCEIK_COMM_ID_BYTES, "RCCL id size");
    if (!id || !mceik_rccl().ok) return 1;
    ncclUniqueId u;
    RCCLCHK(mceik_rccl().GetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return 0;
}

extern "C" int mceik_comm_init(const unsigned char id[MCEIK_COMM_ID_BYTES], int nranks, int rank, int device,
                               mceik_comm **out)
{
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || !mceik_rccl().ok) return 1;
    *out = nullptr;
    DevScope dg(device);
    mceik_comm *c = new mceik_comm();
    c->nranks = nranks; c->rank = rank; c->device = device;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclResult_t r = mceik_rccl().CommInitRank(&c->comm, nranks, u, rank);
    hipError_t e = r == ncclSuccess ? hipMalloc(&c->d_shard, (size_t)nranks * 3 * sizeof(int)) : hipSuccess;
    if (r == ncclSuccess && e == hipSuccess) {
        e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) hipFree(c->d_shard);
    }
    if (r != ncclSuccess || e != hipSuccess) {
        fprintf(stderr, "mceik_comm_init: %s\n", r != ncclSuccess ? mceik_rccl().GetErrorString(r) : hipGetErrorString(e));
        if (r == ncclSuccess) mceik_rccl().CommDestroy(c->comm);
        delete c;
        return -1;
    }
    *out = c;
    return 0;
}

extern "C" int mceik_comm_finalize(mceik_comm **pc)
{
    if (!pc || !*pc) return 0;
    mceik_comm *c = *pc;
    ncclResult_t r;
    {
        DevScope dg(c->device);
        hipStreamSynchronize(c->stream);
        r = mceik_rccl().CommDestroy(c->comm);
        hipStreamDestroy(c->stream);
        hipFree(c->d_shard);
    }
    delete c;
    *pc = nullptr;
    return r == ncclSuccess ? 0 : -1;
}

// Collective.  Every rank's shard [chain_offset, chain_offset + nchains) is
// sent to `root`, which receives it at its global position: point-to-point
// send/recv in one RCCL group (shards may differ in size, no padding), the
// root's own shard by a device copy.  Every rank reaches the all-gather of the
// (offset, count, local status) table whatever fails locally before it (device
// mismatch, a failed sync, the root's staging allocation), and every rank
// decides from the same table, so all return alike and none is left waiting
// in a collective: the first nonzero local status in rank order, else 2 when
// the shards do not tile [0, nchains_total), else the transfer's result.
extern "C" int mceik_mcmc_gather(mceik_mcmc *s, mceik_comm *c, int which, int nchains_total, int root,
                                 int *v_out, double *logl_out)
{
    if (!s || !c || root < 0 || root >= c->nranks || nchains_total < 1) return 1;
    DevScope dg(c->device);
    McmcShard sh;
    const int view = mcmc_shard_view(s, which, &sh);
    const int have = view == 0;
    int status = view < 0 ? -1 : 0;          // -1: the sampler's stream failed or its work queue broke
    if (!status && sh.device != c->device) {
        fprintf(stderr, "mceik_mcmc_gather: sampler on device %d, communicator on %d\n", sh.device, c->device);
        status = 1;
    }
    // A checkpoint is synchronous: the sampler's queued steps have finished
    // (mcmc_shard_view synchronised its stream and checked the work queue),
    // and the gather runs on the communicator's own stream with blocking host
    // copies.
    const size_t ncell = (size_t)sh.ncell;
    const size_t vbytes = (size_t)nchains_total * ncell * sizeof(int), lbytes = (size_t)nchains_total * sizeof(double);
    // root: receive straight into caller device memory on this GPU, else into a
    // staging buffer allocated before the collective starts
    int *d_v = nullptr;
    double *d_l = nullptr;
    bool stage_v = false, stage_l = false;
    if (!status && c->rank == root) {
        stage_v = !on_device(v_out, c->device);
        stage_l = !on_device(logl_out, c->device);
        if (stage_v && hipMalloc((void **)&d_v, vbytes) != hipSuccess) { d_v = nullptr; status = -1; }
        if (!stage_v) d_v = v_out;
        if (!status && stage_l && hipMalloc((void **)&d_l, lbytes) != hipSuccess) { d_l = nullptr; status = -1; }
        if (!stage_l) d_l = logl_out;
        if (status) fprintf(stderr, "mceik_mcmc_gather: cannot allocate the root's staging buffers\n");
    }
    auto release = [&]() {
        if (stage_v && d_v) hipFree(d_v);
        if (stage_l && d_l) hipFree(d_l);
    };
    hipStream_t st = c->stream;
    // 1. every rank learns every shard and status (a rank without a kept state
    // sends count -1)
    const int mine[3] = {sh.chain_offset, have ? sh.nchains : -1, status};
    std::vector<int> all((size_t)c->nranks * 3);
    if (hipMemcpy(c->d_shard + 3 * c->rank, mine, sizeof(mine), hipMemcpyHostToDevice) != hipSuccess ||
        mceik_rccl().AllGather(c->d_shard + 3 * c->rank, c->d_shard, 3, ncclInt32, c->comm, st) != ncclSuccess ||
        hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(all.data(), c->d_shard, all.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) {
        fprintf(stderr, "mceik_mcmc_gather: the shard-table all-gather failed\n");
        release();
        return -1;
    }
    for (int r = 0; r < c->nranks; r++)
        if (all[3 * r + 2]) {
            if (c->rank == root && r != c->rank)
                fprintf(stderr, "mceik_mcmc_gather: rank %d failed locally (%d)\n", r, all[3 * r + 2]);
            release();
            return all[3 * r + 2];
        }
    {   // the shards must tile [0, nchains_total): every rank checks the same table
        int rc = 0;
        std::vector<int> cover((size_t)nchains_total, 0);
        for (int r = 0; r < c->nranks && !rc; r++) {
            const int off = all[3 * r], n = all[3 * r + 1];
            if (n < 0 || off < 0 || (long long)off + n > nchains_total) { rc = 2; break; }
            for (int k = off; k < off + n; k++) cover[k]++;
        }
        for (int k = 0; k < nchains_total && !rc; k++) if (cover[k] != 1) rc = 2;
        if (rc) {
            if (c->rank == root)
                fprintf(stderr, "mceik_mcmc_gather: the ranks' shards (or kept states) do not tile [0, %d)\n",
                        nchains_total);
            release();
            return rc;
        }
    }
    // 2. shards to the root (one RCCL group), the root's own by a device copy
    bool ok = mceik_rccl().GroupStart() == ncclSuccess;
    if (c->rank == root) {
        for (int r = 0; r < c->nranks && ok; r++) {
            if (r == root) continue;
            const size_t off = (size_t)all[3 * r], n = (size_t)all[3 * r + 1];
            ok = mceik_rccl().Recv(d_v + off * ncell, n * ncell, ncclInt32, r, c->comm, st) == ncclSuccess &&
                 mceik_rccl().Recv(d_l + off, n, ncclFloat64, r, c->comm, st) == ncclSuccess;
        }
    } else {
        ok = mceik_rccl().Send(sh.v, (size_t)sh.nchains * ncell, ncclInt32, root, c->comm, st) == ncclSuccess &&
             mceik_rccl().Send(sh.logl, (size_t)sh.nchains, ncclFloat64, root, c->comm, st) == ncclSuccess;
    }
    ok = (mceik_rccl().GroupEnd() == ncclSuccess) && ok;
    if (ok && c->rank == root) {
        const size_t off = (size_t)sh.chain_offset;
        ok = hipMemcpyAsync(d_v + off * ncell, sh.v, (size_t)sh.nchains * ncell * sizeof(int),
                            hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipMemcpyAsync(d_l + off, sh.logl, (size_t)sh.nchains * sizeof(double), hipMemcpyDeviceToDevice,
                            st) == hipSuccess;
    }
    ok = (hipStreamSynchronize(st) == hipSuccess) && ok;
    if (ok && c->rank == root) {
        if (stage_v && v_out) ok = hipMemcpy(v_out, d_v, vbytes, hipMemcpyDeviceToHost) == hipSuccess;
        if (ok && stage_l && logl_out) ok = hipMemcpy(logl_out, d_l, lbytes, hipMemcpyDeviceToHost) == hipSuccess;
    }
    release();
    if (!ok) {
        fprintf(stderr, "mceik_mcmc_gather: RCCL or copy failure\n");
        return -1;
    }
    return 0;
}
