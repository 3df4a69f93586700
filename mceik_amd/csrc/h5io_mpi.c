/* h5io_mpi.c -- the reference's h5io entry points with the reference's own
 * signatures (include/h5io.h; reference h5io.h:18-106, h5io.c), so a
 * homog.c-style MPI harness (homog.c:289-451) links unchanged.
 *
 * The reference runs parallel HDF5: each rank selects its hyperslab
 * {ix0, iy0, iz0} + {nxMax, nyMax, nzMax} of the {nx, ny, nz} dataspace and
 * the ranks write collectively from x-fastest buffers zero-padded to the
 * communicator's largest block (h5io.c:883-925).  The image's HDF5 is serial,
 * so here rank 0 of the communicator owns the file and performs, rank by
 * rank, exactly the selection and H5Dwrite / H5Dread each rank would have
 * issued; the blocks move by MPI gather / scatter (mpi_rt.c, resolved from the
 * caller's MPI at run time).  Every rank returns the same code.  Handles of
 * the other ranks are tagged slots of a table that remembers the grid size.
 */
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MPICH_SKIP_MPICXX 1
#include "../../include/h5io.h"
#include "mpi_rt.h"

/* ---- communicator view (a process without MPI is rank 0 of 1) ---- */
typedef struct {
    int fc, rank, size, mpi;
} Ctx;

static Ctx ctx_of(MPI_Comm comm)
{
    Ctx c;
    c.fc = (int)MPI_Comm_c2f(comm);
    c.rank = mceik_mpi_rank(c.fc);
    c.mpi = c.rank >= 0;
    c.size = c.mpi ? mceik_mpi_size(c.fc) : 1;
    if (!c.mpi || c.size < 1) { c.rank = 0; c.size = 1; c.mpi = 0; }
    return c;
}

/* 0 when no rank failed, else -1 on every rank */
static int agree(const Ctx *c, int rc)
{
    int bad = rc != 0;
    if (c->mpi && mceik_mpi_allreduce_int(c->fc, &bad, 1, 1)) bad = 1;
    return bad ? -1 : 0;
}

/* rank 0's value of an int on every rank */
static int from_root(const Ctx *c, int v)
{
    if (c->mpi) mceik_mpi_bcast_int(c->fc, &v, 1, 0);
    return v;
}

/* ---- handles of ranks other than 0 ---- */
#define REMOTE_TAG ((hid_t)0x4D43454BLL << 32)     /* 'MCEK': no HDF5 id type is this large */
#define REMOTE_MAX 256
static struct { int used, nx, ny, nz; } g_remote[REMOTE_MAX];

static int is_remote(hid_t id) { return (id & ~(hid_t)0xffffffffLL) == REMOTE_TAG; }

static hid_t remote_new(int nx, int ny, int nz)
{
    for (int k = 0; k < REMOTE_MAX; k++)
        if (!g_remote[k].used) {
            g_remote[k].used = 1;
            g_remote[k].nx = nx; g_remote[k].ny = ny; g_remote[k].nz = nz;
            return REMOTE_TAG | (hid_t)k;
        }
    return -1;
}

static int remote_slot(hid_t id)
{
    const int k = (int)(id & 0xffffffffLL);
    return is_remote(id) && k < REMOTE_MAX && g_remote[k].used ? k : -1;
}

/* ---- the blocks: this rank's buffer zero-padded to the max block ---- */
typedef struct {
    int off[3], nmax[3];
} Slab;

/* nmax = the communicator's largest local extent per axis (h5io.c:883-885) */
static int max_extent(const Ctx *c, int nx, int ny, int nz, int nmax[3])
{
    nmax[0] = nx; nmax[1] = ny; nmax[2] = nz;
    return c->mpi ? mceik_mpi_allreduce_int(c->fc, nmax, 3, 1) : 0;
}

static size_t block_elems(const int nmax[3]) { return (size_t)nmax[0] * nmax[1] * nmax[2]; }

/* dense [nz][ny][nx] -> block with nxMax / nyMax strides (h5io.c:894-905) */
static void pack(const float *src, int nx, int ny, int nz, const int nmax[3], float *blk)
{
    memset(blk, 0, block_elems(nmax) * sizeof(float));
    for (int k = 0; k < nz; k++)
        for (int j = 0; j < ny; j++)
            memcpy(blk + ((size_t)k * nmax[1] + j) * nmax[0], src + ((size_t)k * ny + j) * nx, (size_t)nx * 4);
}

static void unpack(const float *blk, int nx, int ny, int nz, const int nmax[3], float *dst)
{
    for (int k = 0; k < nz; k++)
        for (int j = 0; j < ny; j++)
            memcpy(dst + ((size_t)k * ny + j) * nx, blk + ((size_t)k * nmax[1] + j) * nmax[0], (size_t)nx * 4);
}

/* one rank's hyperslab of dataset ds (rank 0 only): the reference's
 * selection and transfer, with a serial transfer property list */
static int slab_io(hid_t ds, const Slab *s, float *blk, int write)
{
    const hsize_t off[3] = {(hsize_t)s->off[0], (hsize_t)s->off[1], (hsize_t)s->off[2]};
    const hsize_t cnt[3] = {1, 1, 1}, stride[3] = {1, 1, 1};
    const hsize_t blkd[3] = {(hsize_t)s->nmax[0], (hsize_t)s->nmax[1], (hsize_t)s->nmax[2]};
    hid_t fsp = H5Dget_space(ds), msp = H5Screate_simple(3, blkd, NULL);
    int rc = fsp < 0 || msp < 0 ? -1 : 0;
    if (rc == 0 && H5Sselect_hyperslab(fsp, H5S_SELECT_SET, off, stride, cnt, blkd) < 0) rc = -1;
    if (rc == 0) {
        herr_t st = write ? H5Dwrite(ds, H5T_NATIVE_FLOAT, msp, fsp, H5P_DEFAULT, blk)
                          : H5Dread(ds, H5T_NATIVE_FLOAT, msp, fsp, H5P_DEFAULT, blk);
        if (st < 0) rc = -1;
    }
    if (msp >= 0) H5Sclose(msp);
    if (fsp >= 0) H5Sclose(fsp);
    return rc;
}

/* Collective write of every rank's padded block `blk` (nmax elements) at its
 * offset into dataset `name` of the file rank 0 holds; rank order. */
static int write_blocks(const Ctx *c, hid_t fid, const char *name, const int off[3], const int nmax[3],
                        const float *blk)
{
    const size_t be = block_elems(nmax), rec = 16 + be * 4;
    char *mine = (char *)malloc(rec), *all = NULL;
    int rc = mine ? 0 : -1;
    if (mine) {
        memset(mine, 0, 16);
        memcpy(mine, off, 3 * sizeof(int));
        memcpy(mine + 16, blk, be * 4);
    }
    if (c->rank == 0) {
        all = c->size > 1 ? (char *)malloc(rec * (size_t)c->size) : mine;
        if (!all) rc = -1;
    }
    if (agree(c, rc)) { free(mine); if (all != mine) free(all); return -1; }
    if (c->size > 1 && mceik_mpi_gather_bytes(c->fc, mine, all, (long long)rec, 0)) rc = -1;
    if (c->rank == 0 && rc == 0) {
        hid_t ds = H5Dopen2(fid, name, H5P_DEFAULT);
        if (ds < 0) rc = -1;
        for (int r = 0; r < c->size && rc == 0; r++) {
            Slab s;
            memcpy(s.off, all + rec * (size_t)r, 3 * sizeof(int));
            memcpy(s.nmax, nmax, sizeof(s.nmax));
            rc = slab_io(ds, &s, (float *)(all + rec * (size_t)r + 16), 1);
        }
        if (ds >= 0) H5Dclose(ds);
    }
    if (all != mine) free(all);
    free(mine);
    return agree(c, rc);
}

/* Collective read: rank 0 reads every rank's hyperslab, each rank gets its block. */
static int read_blocks(const Ctx *c, hid_t fid, const char *name, const int off[3], const int nmax[3], float *blk)
{
    const size_t be = block_elems(nmax), rec = be * 4;
    int *offs = NULL;
    float *all = NULL;
    int rc = 0;
    if (c->rank == 0) {
        offs = (int *)malloc(sizeof(int) * 4 * (size_t)c->size);
        all = (float *)malloc(rec * (size_t)c->size);
        if (!offs || !all) rc = -1;
    }
    if (agree(c, rc)) { free(offs); free(all); return -1; }
    const int mine[4] = {off[0], off[1], off[2], 0};
    if (c->size > 1) {
        if (mceik_mpi_gather_bytes(c->fc, mine, offs, (long long)sizeof(mine), 0)) rc = -1;
    } else {
        memcpy(offs, mine, sizeof(mine));
    }
    if (c->rank == 0 && rc == 0) {
        hid_t ds = H5Dopen2(fid, name, H5P_DEFAULT);
        if (ds < 0) rc = -1;
        for (int r = 0; r < c->size && rc == 0; r++) {
            Slab s;
            memcpy(s.off, offs + 4 * r, 3 * sizeof(int));
            memcpy(s.nmax, nmax, sizeof(s.nmax));
            rc = slab_io(ds, &s, all + be * (size_t)r, 0);
        }
        if (ds >= 0) H5Dclose(ds);
    }
    if (agree(c, rc) == 0) {
        if (c->size > 1) rc = mceik_mpi_scatter_bytes(c->fc, all, blk, (long long)rec, 0);
        else memcpy(blk, all, rec);
    }
    free(offs);
    free(all);
    return agree(c, rc);
}

/* rank 0: does dataset `name` exist?  (every rank learns the answer) */
static int exists_on_root(const Ctx *c, hid_t fid, const char *name, const char *fcnm)
{
    int ok = 0;
    if (c->rank == 0) {
        ok = !is_remote(fid) && H5Lexists(fid, name, H5P_DEFAULT) == 1;
        if (!ok) printf("%s: Error dataset %s doesn't exist\n", fcnm, name);
    }
    return from_root(c, ok);
}

/* write / read of a dense local grid (the reference's public write/read) */
static int write_dense(const Ctx *c, hid_t fid, const char *name, const char *fcnm, int ix0, int iy0, int iz0,
                       int nx, int ny, int nz, const float *src)
{
    if (!exists_on_root(c, fid, name, fcnm)) return -1;
    int nmax[3];
    if (max_extent(c, nx, ny, nz, nmax)) return -1;
    float *blk = (float *)malloc(block_elems(nmax) * sizeof(float) + 4);
    int rc = blk && src ? 0 : -1;
    if (rc == 0) pack(src, nx, ny, nz, nmax, blk);
    if (agree(c, rc)) { free(blk); return -1; }
    const int off[3] = {ix0, iy0, iz0};
    rc = write_blocks(c, fid, name, off, nmax, blk);
    free(blk);
    if (rc && c->rank == 0) printf("%s: Error writing dataset: %s!\n", fcnm, name);
    return rc;
}

static int read_dense(const Ctx *c, hid_t fid, const char *name, const char *fcnm, int ix0, int iy0, int iz0,
                      int nx, int ny, int nz, float *dst)
{
    if (!exists_on_root(c, fid, name, fcnm)) return -1;
    int nmax[3];
    if (max_extent(c, nx, ny, nz, nmax)) return -1;
    float *blk = (float *)malloc(block_elems(nmax) * sizeof(float) + 4);
    int rc = blk && dst ? 0 : -1;
    if (agree(c, rc)) { free(blk); return -1; }
    const int off[3] = {ix0, iy0, iz0};
    rc = read_blocks(c, fid, name, off, nmax, blk);
    if (rc == 0) unpack(blk, nx, ny, nz, nmax, dst);
    else if (c->rank == 0) printf("%s: Error reading dataset %s\n", fcnm, name);
    free(blk);
    return rc;
}

/* rank 0: an empty fp32 dataset with dataspace {nx, ny, nz} */
static int create_dataset(hid_t fid, const char *name, int nx, int ny, int nz)
{
    const hsize_t dims[3] = {(hsize_t)nx, (hsize_t)ny, (hsize_t)nz};
    hid_t sp = H5Screate_simple(3, dims, NULL);
    if (sp < 0) return -1;
    hid_t ds = H5Dcreate2(fid, name, H5T_NATIVE_FLOAT, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    H5Sclose(sp);
    if (ds < 0) return -1;
    return H5Dclose(ds) < 0 ? -1 : 0;
}

static int create_group(hid_t fid, const char *name)
{
    hid_t g = H5Gcreate2(fid, name, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    if (g < 0) return -1;
    return H5Gclose(g) < 0 ? -1 : 0;
}

/* rank 0 creates the file, the others get a slot handle */
static int open_new(const Ctx *c, int job, const char *dirnm, const char *projnm, int nx, int ny, int nz,
                    hid_t *fid, const char *fcnm)
{
    char h5name[PATH_MAX];
    int rc = 0;
    *fid = -1;
    if (c->rank == 0) {
        if (eikonal_h5io_setFileName((enum fileName_enum)job, dirnm, projnm, h5name) != 0) {
            printf("%s: Error setting filename\n", fcnm);
            rc = -1;
        } else {
            *fid = H5Fcreate(h5name, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
            if (*fid < 0) {
                printf("%s: cannot create %s\n", fcnm, h5name);
                rc = -1;
            }
        }
    } else {
        *fid = remote_new(nx, ny, nz);
        if (*fid < 0) rc = -1;
    }
    if (agree(c, rc)) {
        if (c->rank == 0 && *fid >= 0) H5Fclose(*fid);
        else if (remote_slot(*fid) >= 0) g_remote[remote_slot(*fid)].used = 0;
        *fid = -1;
        return -1;
    }
    return 0;
}

int eikonal_h5io_makeModelGroup(const MPI_Comm comm, const hid_t fileID, const int ix0, const int iy0,
                                const int iz0, const int nxGlob, const int nyGlob, const int nzGlob,
                                const int nxLoc, const int nyLoc, const int nzLoc, const int nxMax,
                                const int nyMax, const int nzMax, const double dx, const double dy,
                                const double dz, const double x0, const double y0, const double z0)
{
    const Ctx c = ctx_of(comm);
    static const char *names[3] = {"/Model/xlocs", "/Model/ylocs", "/Model/zlocs"};
    int rc = 0;
    if (c.rank == 0) {
        rc = create_group(fileID, "/Model");
        for (int v = 0; v < 3 && rc == 0; v++) rc = create_dataset(fileID, names[v], nxGlob, nyGlob, nzGlob);
    }
    if (agree(&c, rc)) return -1;
    const int nmax[3] = {nxMax, nyMax, nzMax}, off[3] = {ix0, iy0, iz0};
    float *blk = (float *)calloc(block_elems(nmax) + 1, sizeof(float));
    if (agree(&c, blk ? 0 : -1)) { free(blk); return -1; }
    for (int v = 0; v < 3 && rc == 0; v++) {
        /* this rank's node coordinates in the padded block (h5io.c:453-499) */
        memset(blk, 0, block_elems(nmax) * sizeof(float));
        for (int k = 0; k < nzLoc; k++)
            for (int j = 0; j < nyLoc; j++)
                for (int i = 0; i < nxLoc; i++)
                    blk[((size_t)k * nyMax + j) * nxMax + i] =
                        v == 0 ? (float)(x0 + (double)(i + ix0) * dx)
                               : v == 1 ? (float)(y0 + (double)(j + iy0) * dy) : (float)(z0 + (double)(k + iz0) * dz);
        rc = write_blocks(&c, fileID, names[v], off, nmax, blk);
    }
    free(blk);
    if (rc && c.rank == 0) printf("eikonal_h5io_makeModelGroup: Error writing data!\n");
    return rc;
}

int eikonal_h5io_initTTables(const MPI_Comm comm, const char *dirnm, const char *projnm, const int ix0,
                             const int iy0, const int iz0, const int nx, const int ny, const int nz,
                             const int nxLoc, const int nyLoc, const int nzLoc, const int nmodels,
                             const int nstations, const bool lsaveScratch, const double x0, const double y0,
                             const double z0, const double dx, const double dy, const double dz,
                             hid_t *tttFileID)
{
    const char *fcnm = "eikonal_h5io_initTTables";
    (void)lsaveScratch;                          /* the reference's in-RAM mode is disabled there too (h5io.c:582) */
    const Ctx c = ctx_of(comm);
    if (!tttFileID) return -1;
    int nmax[3];
    if (max_extent(&c, nxLoc, nyLoc, nzLoc, nmax)) return -1;
    if (open_new(&c, TRAVELTIME_FILE, dirnm, projnm, nx, ny, nz, tttFileID, fcnm)) return -1;
    if (eikonal_h5io_makeModelGroup(comm, *tttFileID, ix0, iy0, iz0, nx, ny, nz, nxLoc, nyLoc, nzLoc, nmax[0],
                                    nmax[1], nmax[2], dx, dy, dz, x0, y0, z0) != 0) {
        if (c.rank == 0) printf("%s: Error making model group\n", fcnm);
        return -1;
    }
    int rc = 0;
    char name[512];
    if (c.rank == 0) {
        rc = create_group(*tttFileID, "/TravelTimeTables");
        for (int m = 1; m <= nmodels && rc == 0; m++) {
            snprintf(name, sizeof(name), "/TravelTimeTables/Model_%d", m);
            rc = create_group(*tttFileID, name);
            for (int s = 1; s <= nstations && rc == 0; s++) {
                snprintf(name, sizeof(name), "/TravelTimeTables/Model_%d/Station_%d", m, s);
                rc = create_group(*tttFileID, name);
                for (int ph = 1; ph <= 2 && rc == 0; ph++) {
                    eikonal_h5io_setTravelTimeName(m, s, ph == 1, name);
                    rc = create_dataset(*tttFileID, name, nx, ny, nz);
                }
            }
        }
        if (rc) printf("%s: Failed to create the table groups\n", fcnm);
    }
    if (agree(&c, rc)) return -1;
    /* the null tables (h5io.c:685-709) */
    float *zero = (float *)calloc((size_t)nxLoc * nyLoc * nzLoc + 1, sizeof(float));
    if (agree(&c, zero ? 0 : -1)) { free(zero); return -1; }
    for (int m = 1; m <= nmodels && rc == 0; m++)
        for (int s = 1; s <= nstations && rc == 0; s++)
            for (int ph = 1; ph <= 2 && rc == 0; ph++)
                rc = eikonal_h5io_writeTravelTimes(comm, *tttFileID, s, m, ph, ix0, iy0, iz0, nxLoc, nyLoc, nzLoc,
                                                   zero);
    free(zero);
    if (rc && c.rank == 0) printf("%s: Error writing null ttimes\n", fcnm);
    return rc;
}

int eikonal_h5io_initLocations(const MPI_Comm comm, const char *dirnm, const char *projnm, const int ix0,
                               const int iy0, const int iz0, const int nx, const int ny, const int nz,
                               const int nxLoc, const int nyLoc, const int nzLoc, const int nmodels,
                               const int nevents, const double x0, const double y0, const double z0,
                               const double dx, const double dy, const double dz, hid_t *locFileID)
{
    const char *fcnm = "eikonal_h5io_initLocations";
    const Ctx c = ctx_of(comm);
    if (!locFileID) return -1;
    int nmax[3];
    if (max_extent(&c, nxLoc, nyLoc, nzLoc, nmax)) return -1;
    if (open_new(&c, LOCATION_FILE, dirnm, projnm, nx, ny, nz, locFileID, fcnm)) return -1;
    if (eikonal_h5io_makeModelGroup(comm, *locFileID, ix0, iy0, iz0, nx, ny, nz, nxLoc, nyLoc, nzLoc, nmax[0],
                                    nmax[1], nmax[2], dx, dy, dz, x0, y0, z0) != 0) {
        if (c.rank == 0) printf("%s: Error making model group\n", fcnm);
        return -1;
    }
    /* the uniform prior: the whole padded block is 1 (h5io.c:309-313) */
    int rc = c.rank == 0 ? create_dataset(*locFileID, "/Model/priorLocationModel", nx, ny, nz) : 0;
    if (agree(&c, rc)) return -1;
    const size_t be = block_elems(nmax);
    float *one = (float *)malloc((be + 1) * sizeof(float));
    if (agree(&c, one ? 0 : -1)) { free(one); return -1; }
    for (size_t i = 0; i < be; i++) one[i] = 1.0f;
    const int off[3] = {ix0, iy0, iz0};
    rc = write_blocks(&c, *locFileID, "/Model/priorLocationModel", off, nmax, one);
    free(one);
    if (rc) {
        if (c.rank == 0) printf("%s: Error writing prior!\n", fcnm);
        return -1;
    }
    char name[512];
    if (c.rank == 0) {
        rc = create_group(*locFileID, "/logJPDFs");
        for (int e = 1; e <= nevents && rc == 0; e++) {
            snprintf(name, sizeof(name), "/logJPDFs/Event_%d", e);
            rc = create_group(*locFileID, name);
            for (int m = 1; m <= nmodels && rc == 0; m++) {
                snprintf(name, sizeof(name), "/logJPDFs/Event_%d/Model_%d", e, m);
                rc = create_group(*locFileID, name);
                eikonal_h5io_setLocationName(m, e, name);
                if (rc == 0) rc = create_dataset(*locFileID, name, nx, ny, nz);
            }
        }
        if (rc) printf("%s: Error making model group\n", fcnm);
    }
    if (agree(&c, rc)) return -1;
    float *zero = (float *)calloc((size_t)nxLoc * nyLoc * nzLoc + 1, sizeof(float));
    if (agree(&c, zero ? 0 : -1)) { free(zero); return -1; }
    for (int e = 1; e <= nevents && rc == 0; e++)
        for (int m = 1; m <= nmodels && rc == 0; m++)
            rc = eikonal_h5io_writeLocationLogJPDF(comm, *locFileID, m, e, ix0, iy0, iz0, nxLoc, nyLoc, nzLoc, zero);
    free(zero);
    if (rc && c.rank == 0) printf("%s: Error writing null jpdfs\n", fcnm);
    return rc;
}

int eikonal_h5io_writeTravelTimes(const MPI_Comm comm, const hid_t tttFileID, const int station,
                                  const int model, const int iphase, const int ix0, const int iy0,
                                  const int iz0, const int nxLoc, const int nyLoc, const int nzLoc,
                                  const float *__restrict__ ttimes)
{
    char name[512];
    const Ctx c = ctx_of(comm);
    eikonal_h5io_setTravelTimeName(model, station, iphase != 2, name);
    return write_dense(&c, tttFileID, name, "eikonal_h5io_writeTravelTimes", ix0, iy0, iz0, nxLoc, nyLoc, nzLoc,
                       ttimes);
}

int eikonal_h5io_readTravelTimes(const MPI_Comm comm, const hid_t tttFileID, const int station,
                                 const int model, const int iphase, const int ix0, const int iy0,
                                 const int iz0, const int nxLoc, const int nyLoc, const int nzLoc,
                                 float *__restrict__ ttimes)
{
    char name[512];
    const Ctx c = ctx_of(comm);
    eikonal_h5io_setTravelTimeName(model, station, iphase != 2, name);
    return read_dense(&c, tttFileID, name, "eikonal_h5io_readTravelTimes", ix0, iy0, iz0, nxLoc, nyLoc, nzLoc,
                      ttimes);
}

int eikonal_h5io_writeLocationLogJPDF(const MPI_Comm comm, const hid_t locFileID, const int model,
                                      const int event, const int ix0, const int iy0, const int iz0,
                                      const int nxLoc, const int nyLoc, const int nzLoc,
                                      const float *__restrict__ logJPDF)
{
    char name[512];
    const Ctx c = ctx_of(comm);
    eikonal_h5io_setLocationName(model, event, name);
    return write_dense(&c, locFileID, name, "eikonal_h5io_writeLocationLogJPDF", ix0, iy0, iz0, nxLoc, nyLoc,
                       nzLoc, logJPDF);
}

int eikonal_h5io_readModel(const MPI_Comm comm, const hid_t fileID, const int ix0, const int iy0,
                           const int iz0, const int nxLoc, const int nyLoc, const int nzLoc,
                           float *__restrict__ xlocs, float *__restrict__ ylocs, float *__restrict__ zlocs)
{
    const Ctx c = ctx_of(comm);
    static const char *names[3] = {"/Model/xlocs", "/Model/ylocs", "/Model/zlocs"};
    float *dst[3] = {xlocs, ylocs, zlocs};
    for (int v = 0; v < 3; v++)
        if (read_dense(&c, fileID, names[v], "eikonal_h5io_readModel", ix0, iy0, iz0, nxLoc, nyLoc, nzLoc, dst[v]))
            return -1;
    return 0;
}

int eikonal_h5io_getModelDimensions(const hid_t fileID, int *nx, int *ny, int *nz)
{
    const char *fcnm = "eikonal_h5io_getModelDimensions";
    *nx = *ny = *nz = 0;
    const int k = remote_slot(fileID);
    if (k >= 0) {                                  /* a non-root rank's handle */
        *nx = g_remote[k].nx; *ny = g_remote[k].ny; *nz = g_remote[k].nz;
        return 0;
    }
    if (H5Lexists(fileID, "/Model/xlocs", H5P_DEFAULT) != 1) {
        printf("%s: Error dataset /Model/xlocs doesn't exist\n", fcnm);
        return -1;
    }
    hid_t ds = H5Dopen2(fileID, "/Model/xlocs", H5P_DEFAULT);
    hid_t sp = H5Dget_space(ds);
    const int rank = H5Sget_simple_extent_ndims(sp);
    hsize_t dims[3] = {0, 0, 0};
    int rc = 0;
    if (rank < 1 || rank > 3 || H5Sget_simple_extent_dims(sp, dims, NULL) < 0) {
        printf("%s: Invalid rank %d\n", fcnm, rank);
        rc = -1;
    } else if (rank == 1) {                        /* unstructured: one count (h5io.c:143-149) */
        *nx = *ny = *nz = (int)dims[0];
    } else {
        *nx = (int)dims[0]; *ny = (int)dims[1]; *nz = (int)dims[2];
    }
    H5Sclose(sp);
    H5Dclose(ds);
    return rc;
}

int eikonal_h5io_finalize(const MPI_Comm comm, hid_t *tttFileID)
{
    (void)comm;
    if (!tttFileID) return -1;
    const int k = remote_slot(*tttFileID);
    if (k >= 0) {
        g_remote[k].used = 0;
        return 0;
    }
    if (H5Fclose(*tttFileID) < 0) {
        printf("eikonal_h5io_finalize: Failed closing travel time table file\n");
        return -1;
    }
    return 0;
}

/* ---- Fortran interfaces (1-based offsets, h5io.c:76-89, 960-987, 1162-1193) ---- */
void eikonal_h5io_getModelDimensionsF(const long *inFileID, int *nx, int *ny, int *nz, int *ierr)
{
    *ierr = eikonal_h5io_getModelDimensions((hid_t)*inFileID, nx, ny, nz) != 0 ? 1 : 0;
    if (*ierr) printf("eikonal_h5io_getModelDimensionsF: Error getting dimensions\n");
}

void eikonal_h5io_readModelF(const int *comm, const long *inFileID, const int *ix0, const int *iy0,
                             const int *iz0, const int *nxLoc, const int *nyLoc, const int *nzLoc,
                             float *__restrict__ xlocs, float *__restrict__ ylocs, float *__restrict__ zlocs,
                             int *ierr)
{
    *ierr = eikonal_h5io_readModel(MPI_Comm_f2c(*comm), (hid_t)*inFileID, *ix0 - 1, *iy0 - 1, *iz0 - 1, *nxLoc,
                                   *nyLoc, *nzLoc, xlocs, ylocs, zlocs) != 0 ? 1 : 0;
    if (*ierr) printf("eikonal_h5io_readModelF: Error reading model\n");
}

void eikonal_h5io_readTraveltimesF(const int *comm, const long *tttFileID, const int *station,
                                   const int *model, const int *iphase, const int *ix0f, const int *iy0f,
                                   const int *iz0f, const int *nxLoc, const int *nyLoc, const int *nzLoc,
                                   float *ttimes, int *ierr)
{
    *ierr = eikonal_h5io_readTravelTimes(MPI_Comm_f2c(*comm), (hid_t)*tttFileID, *station, *model, *iphase,
                                         *ix0f - 1, *iy0f - 1, *iz0f - 1, *nxLoc, *nyLoc, *nzLoc, ttimes) != 0;
    if (*ierr) {
        printf("eikonal_h5io_readTraveltimesF: Error calling eikonal_h5io_readTravelTimes\n");
        memset(ttimes, 0, (size_t)(*nxLoc) * (*nyLoc) * (*nzLoc) * sizeof(float));
    }
}
