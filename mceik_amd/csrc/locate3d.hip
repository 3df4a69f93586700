// locate3d.hip -- the reference's MPI location driver entry points
// (include/locate.h; reference locate.f90:322-689, include/locate.h:10-23),
// host code over the batched GPU relocation (capi.hip mceik_relocate).
//
// locate3d_initialize follows LOCATE3D_INITIALIZE (locate.f90:562-677): the
// master reads the model dimensions from the travel-time file and broadcasts
// them with the block decomposition, the intra-table communicator is split by
// mpiutils_initialize3d if the harness has not done it, every rank takes its
// block (MPIUTILS_GRD2IJK, ndx = max(n / ndiv, 1), the last block to the grid
// end), the blocks must tile the grid, and the rank reads its block of
// /Model/{x,y,z}locs.  locate3d_gridsearch replaces LOCATE3D_GRIDSEARCH's
// per-observation HDF5 reads and fp64 stacking (locate.f90:385-500) by one
// read per distinct (station, phase) table of the block and one
// mceik_relocate launch (every event, every node; locate.c's fp32 L2 with the
// analytic origin time, the weighting SURVEY s.8a row a12 chose), then the
// MAXLOC over the block and over the blocks in block order (locate.f90:
// 469-498).  Deviations: include/locate.h.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/locate.h"
#include "../../include/mceik_eikonal.h"
#include "../../include/mpiutils.h"
#include "mpi_rt.h"

extern "C" MCEIK_HIDDEN int mceik_mpiutils_initialized(void);

namespace {

// the library's h5io entry points (libmceik_h5io.so), the Fortran-handle forms
// (no MPI or HDF5 types cross this boundary), resolved at run time
struct H5io {
    void (*dims)(const long *, int *, int *, int *, int *) = nullptr;
    void (*model)(const int *, const long *, const int *, const int *, const int *, const int *, const int *,
                  const int *, float *, float *, float *, int *) = nullptr;
    void (*ttimes)(const int *, const long *, const int *, const int *, const int *, const int *, const int *,
                   const int *, const int *, const int *, const int *, float *, int *) = nullptr;
    bool ok() const { return dims && model && ttimes; }
};

const H5io &h5io()
{
    static H5io h = [] {
        H5io x;
        auto bind = [&](void *lib) {
            x.dims = reinterpret_cast<decltype(x.dims)>(dlsym(lib, "eikonal_h5io_getModelDimensionsF"));
            x.model = reinterpret_cast<decltype(x.model)>(dlsym(lib, "eikonal_h5io_readModelF"));
            x.ttimes = reinterpret_cast<decltype(x.ttimes)>(dlsym(lib, "eikonal_h5io_readTraveltimesF"));
        };
        bind(RTLD_DEFAULT);                 // the harness linked libmceik_h5io.so
        if (!x.ok()) {                      // else the one next to this library
            Dl_info di;
            if (dladdr(reinterpret_cast<void *>(&locate3d_finalize), &di) && di.dli_fname) {
                std::string p(di.dli_fname);
                const size_t s = p.rfind('/');
                p = (s == std::string::npos ? std::string() : p.substr(0, s + 1)) + "libmceik_h5io.so";
                if (void *lib = dlopen(p.c_str(), RTLD_NOW | RTLD_GLOBAL)) bind(lib);
            }
        }
        if (!x.ok()) fprintf(stderr, "locate3d: the h5io entry points (libmceik_h5io.so) are not available\n");
        return x;
    }();
    return h;
}

// LOCATE_MODULE's parms and locate (module.F90) for this rank
struct Locator {
    bool init = false;
    int iverb = 0, nx = 0, ny = 0, nz = 0, ndivx = 1, ndivy = 1, ndivz = 1;
    long ttt = 0, loc = 0;
    int comm = 0;                        // intra-table communicator (Fortran handle), or the caller's
    bool mpi = false;                    // the process runs MPI
    int ix0 = 1, iy0 = 1, iz0 = 1;       // 1-based block origin
    int nxLoc = 0, nyLoc = 0, nzLoc = 0;
    std::vector<float> xlocs, ylocs, zlocs;
    long long ngrd() const { return (long long)nxLoc * nyLoc * nzLoc; }
};
Locator g_loc;

int rank_of(const Locator &s) { return s.mpi ? mceik_mpi_rank(s.comm) : 0; }
int size_of(const Locator &s) { return s.mpi ? mceik_mpi_size(s.comm) : 1; }

#define LHIP(x)                                                                          \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "locate3d_gridsearch: %s: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

// The relocation of this rank's block: tables read once per distinct
// (station, phase), one mceik_relocate launch for job 2 (one per event for
// job 1, t0 = tori), MAXLOC per event.  best [nevents][5 + nobs]: the
// block's best node (log-PDF, x, y, z, t0) and the table values there of the
// event's observations, as exchanged between the blocks.
int block_search(const Locator &s, int model, int job, int nobs, int nev, const int *luse, const int *stat,
                 const int *ptype, const double *statCor, const double *tori, const double *varobs,
                 const double *tobs, std::vector<double> &best)
{
    const long long ngrd = s.ngrd();
    const int w = 5 + nobs;
    best.assign((size_t)nev * w, 0.0);
    for (int e = 0; e < nev; e++) best[(size_t)e * w] = -HUGE_VAL;   // (an empty block never wins)
    // distinct tables in first-use order (every rank of the intra-table communicator reads them in the
    // same order: the reads are collective)
    std::map<std::pair<int, int>, int> rowof;
    std::vector<std::pair<int, int>> rows;
    for (int e = 0; e < nev; e++)
        for (int i = 0; i < nobs; i++) {
            const size_t k = (size_t)e * nobs + i;
            if (!luse[k]) continue;
            const std::pair<int, int> key(stat[k], ptype[k]);
            if (!rowof.count(key)) {
                rowof[key] = (int)rows.size();
                rows.push_back(key);
            }
        }
    std::vector<float> tab((size_t)std::max<size_t>(rows.size(), 1) * ngrd);
    int rerr = 0;
    for (size_t r = 0; r < rows.size(); r++) {
        int ierr = 0;
        h5io().ttimes(&s.comm, &s.ttt, &rows[r].first, &model, &rows[r].second, &s.ix0, &s.iy0, &s.iz0, &s.nxLoc,
                      &s.nyLoc, &s.nzLoc, tab.data() + r * ngrd, &ierr);
        rerr |= ierr;
    }
    if (rerr) {
        fprintf(stderr, "locate3d_gridsearch: Error reading observed traveltimes\n");
        return 1;
    }
    // compacted observations per event (eikonal.relocate's packing: fp32 tobs - tcorr, 1/var, the
    // running fp32 sum of the weights)
    std::vector<int> ptr(1, 0), orow;
    std::vector<float> tc, wt, xn;
    for (int e = 0; e < nev; e++) {
        float x = 0.0f;
        for (int i = 0; i < nobs; i++) {
            const size_t k = (size_t)e * nobs + i;
            if (!luse[k]) continue;
            orow.push_back(rowof[std::make_pair(stat[k], ptype[k])]);
            tc.push_back((float)tobs[k] - (float)statCor[i]);
            const float wi = 1.0f / (float)varobs[k];
            wt.push_back(wi);
            x = x + wi;
        }
        xn.push_back(x);
        ptr.push_back((int)orow.size());
    }
    if (ngrd == 0) return 0;
    const int nused = (int)orow.size();
    float *d_tab = nullptr, *d_tc = nullptr, *d_wt = nullptr, *d_xn = nullptr, *d_out = nullptr, *d_t0 = nullptr;
    int *d_ptr = nullptr, *d_row = nullptr;
    const size_t ob = (size_t)std::max(nused, 1);
    LHIP(hipMalloc(&d_tab, tab.size() * 4));
    LHIP(hipMalloc(&d_ptr, ptr.size() * 4));
    LHIP(hipMalloc(&d_row, ob * 4));
    LHIP(hipMalloc(&d_tc, ob * 4));
    LHIP(hipMalloc(&d_wt, ob * 4));
    LHIP(hipMalloc(&d_xn, (size_t)nev * 4));
    LHIP(hipMalloc(&d_out, (size_t)nev * ngrd * 4));
    LHIP(hipMalloc(&d_t0, (size_t)nev * ngrd * 4));
    LHIP(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    LHIP(hipMemcpy(d_ptr, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice));
    if (nused) {
        LHIP(hipMemcpy(d_row, orow.data(), (size_t)nused * 4, hipMemcpyHostToDevice));
        LHIP(hipMemcpy(d_tc, tc.data(), (size_t)nused * 4, hipMemcpyHostToDevice));
        LHIP(hipMemcpy(d_wt, wt.data(), (size_t)nused * 4, hipMemcpyHostToDevice));
    }
    LHIP(hipMemcpy(d_xn, xn.data(), (size_t)nev * 4, hipMemcpyHostToDevice));
    int rc = 0;
    // job 2: every event in one single-pass launch; job 1: one launch per event (its own t0)
    auto launch = [&](int e0, int ne, int want_ot, float t0use) {
        mceik_relocate_batch b;
        memset(&b, 0, sizeof(b));
        b.ldgrd = (int)ngrd; b.ngrd = (int)ngrd; b.nev = ne; b.iwantOT = want_ot; b.t0use = t0use;
        b.tables = d_tab; b.ev_ptr = d_ptr + e0; b.obs_row = d_row; b.tc = d_tc; b.wt = d_wt; b.xnorm = d_xn + e0;
        b.t0 = d_t0 + (size_t)e0 * ngrd; b.out = d_out + (size_t)e0 * ngrd; b.log_pdf = 1;
        // (single pass when the launch covers every event; a per-event launch offsets ev_ptr into the
        // shared arrays, which the two-pass kernel takes)
        b.nrows = ne == nev ? (int)rows.size() : 0;
        b.nobs = ne == nev ? nused : 0;
        if (mceik_relocate(&b, nullptr) != 0) rc = 1;
    };
    if (job == 2) {
        launch(0, nev, 1, 0.0f);
    } else {
        for (int e = 0; e < nev; e++) launch(e, 1, 0, (float)tori[e]);
    }
    std::vector<float> out((size_t)nev * ngrd), t0((size_t)nev * ngrd);
    if (!rc) {
        LHIP(hipDeviceSynchronize());
        LHIP(hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost));
        LHIP(hipMemcpy(t0.data(), d_t0, t0.size() * 4, hipMemcpyDeviceToHost));
    }
    hipFree(d_tab); hipFree(d_ptr); hipFree(d_row); hipFree(d_tc); hipFree(d_wt); hipFree(d_xn);
    hipFree(d_out); hipFree(d_t0);
    if (rc) {
        fprintf(stderr, "locate3d_gridsearch: mceik_relocate failed\n");
        return 1;
    }
    for (int e = 0; e < nev; e++) {
        const float *o = out.data() + (size_t)e * ngrd;
        long long g = 0;                                     // MAXLOC: the first largest log-PDF
        for (long long j = 1; j < ngrd; j++)
            if (o[j] > o[g]) g = j;
        double *bst = best.data() + (size_t)e * w;
        bst[0] = o[g];
        bst[1] = s.xlocs[g]; bst[2] = s.ylocs[g]; bst[3] = s.zlocs[g];
        bst[4] = job == 2 ? (double)t0[(size_t)e * ngrd + g] : tori[e];
        for (int i = 0; i < nobs; i++) {
            const size_t k = (size_t)e * nobs + i;
            bst[5 + i] = luse[k] ? (double)tab[(size_t)rowof[std::make_pair(stat[k], ptype[k])] * ngrd + g] : 0.0;
        }
    }
    return 0;
}

}  // namespace

extern "C" void locate3d_initialize(const int *comm, const int *iverb, const long *tttFileID, const long *locFileID,
                                    const int *ndivx, const int *ndivy, const int *ndivz, int *ierr)
{
    *ierr = 0;
    Locator s;
    s.mpi = mceik_mpi_rank(*comm) >= 0;
    s.comm = *comm;
    const int myid = rank_of(s);
    if (!h5io().ok()) {
        *ierr = 1;
        return;
    }
    int p[8] = {0, 0, 0, 0, *ndivx, *ndivy, *ndivz, 0};
    if (myid == 0) {
        int e = 0;
        h5io().dims(tttFileID, &p[1], &p[2], &p[3], &e);
        if (e != 0) printf("locate3d_initialize: Error getting dimensions\n");
        p[0] = *iverb;
        p[7] = e != 0;
    }
    if (s.mpi) mceik_mpi_bcast_int(s.comm, p, 8, 0);   // the master's parameters (locate.f90:601-609)
    s.iverb = p[0]; s.nx = p[1]; s.ny = p[2]; s.nz = p[3]; s.ndivx = p[4]; s.ndivy = p[5]; s.ndivz = p[6];
    s.ttt = *tttFileID; s.loc = *locFileID;             // (each rank keeps its own h5io handles)
    if (p[7] || s.ndivx < 1 || s.ndivy < 1 || s.ndivz < 1) {
        *ierr = 1;
        return;
    }
    if (s.mpi && !mceik_mpiutils_initialized()) {
        printf("locate_initialize3d: Splitting communicator...\n");
        const int ireord = 1, iwt = 0;
        mpiutils_initialize3d(comm, &ireord, &iwt, &s.ndivx, &s.ndivy, &s.ndivz, ierr);
        if (*ierr != 0) {
            printf("locate_initialize3d: Error splitting communicator\n");
            *ierr = 1;
            return;
        }
    }
    if (s.mpi) {                                         // the reads are collective over the table's ranks
        int g = 0, intra = 0, inter = 0, e = 0;
        mpiutils_getCommunicators(&g, &intra, &inter, &e);
        if (!e) s.comm = intra;
    }
    const int blk = rank_of(s);
    int imbx = 0, imby = 0, imbz = 0, e = 0;
    mpiutils_grd2ijk(&blk, &s.ndivx, &s.ndivy, &s.ndivz, &imbx, &imby, &imbz, &e);
    if (e != 0) {
        printf("Error finding process block\n");
        *ierr = 1;
        return;
    }
    const int ndx = std::max(s.nx / s.ndivx, 1), ndy = std::max(s.ny / s.ndivy, 1), ndz = std::max(s.nz / s.ndivz, 1);
    int i1 = ndx * imbx + 1, i2 = ndx * (imbx + 1), j1 = ndy * imby + 1, j2 = ndy * (imby + 1);
    int k1 = ndz * imbz + 1, k2 = ndz * (imbz + 1);
    if (imbx + 1 == s.ndivx) i2 = s.nx;
    if (imby + 1 == s.ndivy) j2 = s.ny;
    if (imbz + 1 == s.ndivz) k2 = s.nz;
    s.nxLoc = std::max(i2 - i1 + 1, 0); s.nyLoc = std::max(j2 - j1 + 1, 0); s.nzLoc = std::max(k2 - k1 + 1, 0);
    s.ix0 = i1; s.iy0 = j1; s.iz0 = k1;
    // the blocks must tile the grid (locate.f90:651-658; every rank learns the answer here)
    int ng = (int)s.ngrd();
    if (s.mpi) mceik_mpi_allreduce_int(s.comm, &ng, 1, 0);
    if ((long long)ng != (long long)s.nx * s.ny * s.nz) {
        if (myid == 0) printf("locate3d_initialize: Failed to split grid %lld %d\n", (long long)s.nx * s.ny * s.nz, ng);
        *ierr = 1;
    }
    const size_t n = (size_t)std::max<long long>(s.ngrd(), 1);
    s.xlocs.assign(n, 0.0f); s.ylocs.assign(n, 0.0f); s.zlocs.assign(n, 0.0f);
    int re = 0;
    h5io().model(&s.comm, tttFileID, &s.ix0, &s.iy0, &s.iz0, &s.nxLoc, &s.nyLoc, &s.nzLoc, s.xlocs.data(),
                 s.ylocs.data(), s.zlocs.data(), &re);
    if (re != 0) {
        printf("locate3d_initialize: Error reading model\n");
        *ierr = 1;
    }
    s.init = true;
    g_loc = std::move(s);
}

extern "C" void locate3d_gridsearch(const int *model, const int *job, const int *nobs, const int *nevents,
                                    const int *luseObs, const int *statPtr, const int *pickType,
                                    const double *statCor, const double *tori, const double *varobs,
                                    const double *tobs, double *test, double *hypo, int *ierr)
{
    *ierr = 0;
    const Locator &s = g_loc;
    if (!s.init) {
        printf("locate3d_gridsearch: locate3d_initialize was not called\n");
        *ierr = 1;
        return;
    }
    if (*job == 3 || *job == 5) {                        // COMPUTE_LOCATION_AND_STATICS / _ALL
        printf(" Not yet done\n");
        *ierr = 1;
        return;
    }
    if (*job != 1 && *job != 2) {
        printf(" locate_gridsearch: Invalid job\n");
        *ierr = 1;
        return;
    }
    const int nob = *nobs, nev = *nevents, w = 5 + nob;
    if (nob < 0 || nev < 0) {
        *ierr = 1;
        return;
    }
    std::vector<double> best;
    int bad = block_search(s, *model, *job, nob, nev, luseObs, statPtr, pickType, statCor, tori, varobs, tobs, best);
    // the blocks agree on failure, then on the hypocentres: the first block holding the largest
    // log-PDF (locate.f90:470-498's ALLREDUCE MAX + MAXLOC)
    const int nb = size_of(s);
    if (s.mpi) mceik_mpi_allreduce_int(s.comm, &bad, 1, 1);
    if (bad) {
        *ierr = 1;
        return;
    }
    std::vector<double> all((size_t)nb * best.size());
    if (s.mpi && nb > 1) {
        if (mceik_mpi_allgather_bytes(s.comm, best.data(), all.data(), (int)(best.size() * sizeof(double))) != 0) {
            *ierr = 1;
            return;
        }
    } else {
        all = best;
    }
    for (int e = 0; e < nev; e++) {
        int ib = 0;
        for (int b = 1; b < nb; b++)
            if (all[((size_t)b * nev + e) * w] > all[((size_t)ib * nev + e) * w]) ib = b;
        const double *bst = all.data() + ((size_t)ib * nev + e) * w;
        for (int c = 0; c < 4; c++) hypo[4 * e + c] = bst[1 + c];
        for (int i = 0; i < nob; i++) {
            const size_t k = (size_t)e * nob + i;
            if (luseObs[k]) test[k] = bst[4] + bst[5 + i];
        }
        if (s.iverb > 0 && rank_of(s) == 0)
            printf("locate3d_gridsearch: event %d block %d logPDF %.9g hypo %g %g %g %g\n", e + 1, ib, bst[0],
                   hypo[4 * e], hypo[4 * e + 1], hypo[4 * e + 2], hypo[4 * e + 3]);
    }
}

extern "C" void locate3d_finalize(void)
{
    g_loc = Locator();
}
