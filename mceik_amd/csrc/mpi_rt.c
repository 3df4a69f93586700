/* mpi_rt.c -- the MPI calls of the MPI-variant drop-in (eikonal3d_initialize /
 * solve / finalize, fsm3d.f90:1583-1929), resolved at run time.
 *
 * The reference's MPI variant is collective over `comm`: the master
 * broadcasts the solver parameters (fsm3d.f90:1626-1639) and the SETBCS
 * error (:1792), so every rank returns the master's ierr.  The library keeps
 * no link dependency on MPI: when the calling process has MPI loaded (an MPI
 * main linked with libmpi, or mpi4py) and initialised, the symbols are taken
 * from it (dlsym RTLD_DEFAULT, else an already-loaded libmpi.so.12 via
 * RTLD_NOLOAD); otherwise the caller is a single process and these return -1
 * ("no MPI"), the drop-in then acting as rank 0 of one.  Built against the
 * image's MPICH mpi.h (the MPI the reference builds with); without it the
 * file compiles to the no-MPI answers.  Internal: not part of include/. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpi_rt.h"

#if defined(__has_include)
#if __has_include(<mpi.h>)
#define MPICH_SKIP_MPICXX 1
#include <mpi.h>
#define MCEIK_HAVE_MPI_H 1
#endif
#endif

#ifdef MCEIK_HAVE_MPI_H
typedef int (*flag_fn)(int *);
typedef int (*rank_fn)(MPI_Comm, int *);
typedef int (*bcast_fn)(void *, int, MPI_Datatype, int, MPI_Comm);
typedef int (*allreduce_fn)(const void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm);
typedef int (*allgather_fn)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPI_Comm);
typedef int (*isend_fn)(const void *, int, MPI_Datatype, int, int, MPI_Comm, MPI_Request *);
typedef int (*irecv_fn)(void *, int, MPI_Datatype, int, int, MPI_Comm, MPI_Request *);
typedef int (*waitall_fn)(int, MPI_Request *, MPI_Status *);
typedef int (*gather_fn)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, int, MPI_Comm);
typedef int (*scatter_fn)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, int, MPI_Comm);
typedef int (*barrier_fn)(MPI_Comm);
typedef int (*dup_fn)(MPI_Comm, MPI_Comm *);
typedef int (*split_fn)(MPI_Comm, int, int, MPI_Comm *);
typedef int (*free_fn)(MPI_Comm *);

static struct {
    int tried, ok;
    flag_fn initialized, finalized;
    rank_fn rank, size;
    bcast_fn bcast;
    allreduce_fn allreduce;
    allgather_fn allgather;
    isend_fn isend;
    irecv_fn irecv;
    waitall_fn waitall;
    gather_fn gather;
    scatter_fn scatter;
    barrier_fn barrier;
    dup_fn dup;
    split_fn split;
    free_fn cfree;
} rt;

static void *sym(void *h, const char *name)
{
    void *p = dlsym(RTLD_DEFAULT, name);
    return p ? p : (h ? dlsym(h, name) : NULL);
}

static int load(void)
{
    if (!rt.tried) {
        rt.tried = 1;
        void *h = dlopen("libmpi.so.12", RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
        if (!h) h = dlopen("libmpi.so", RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
        rt.initialized = (flag_fn)sym(h, "MPI_Initialized");
        rt.finalized = (flag_fn)sym(h, "MPI_Finalized");
        rt.rank = (rank_fn)sym(h, "MPI_Comm_rank");
        rt.size = (rank_fn)sym(h, "MPI_Comm_size");
        rt.bcast = (bcast_fn)sym(h, "MPI_Bcast");
        rt.allreduce = (allreduce_fn)sym(h, "MPI_Allreduce");
        rt.allgather = (allgather_fn)sym(h, "MPI_Allgather");
        rt.isend = (isend_fn)sym(h, "MPI_Isend");
        rt.irecv = (irecv_fn)sym(h, "MPI_Irecv");
        rt.waitall = (waitall_fn)sym(h, "MPI_Waitall");
        rt.gather = (gather_fn)sym(h, "MPI_Gather");
        rt.scatter = (scatter_fn)sym(h, "MPI_Scatter");
        rt.barrier = (barrier_fn)sym(h, "MPI_Barrier");
        rt.dup = (dup_fn)sym(h, "MPI_Comm_dup");
        rt.split = (split_fn)sym(h, "MPI_Comm_split");
        rt.cfree = (free_fn)sym(h, "MPI_Comm_free");
        rt.ok = rt.initialized && rt.finalized && rt.rank && rt.size && rt.bcast && rt.allreduce && rt.allgather &&
                rt.isend && rt.irecv && rt.waitall && rt.gather && rt.scatter && rt.barrier && rt.dup && rt.split &&
                rt.cfree;
        // The handles passed below (MPI_INT, MPI_DOUBLE, MPI_IN_PLACE,
        // MPI_Comm_f2c) are MPICH-ABI compile-time constants: an MPI of
        // another ABI (Open MPI, e.g. through mpi4py or torch) would take them
        // as pointers.  Only an MPICH-ABI library is used; any other counts
        // as no MPI, said once.
        typedef int (*libver_fn)(char *, int *);
        libver_fn ver = (libver_fn)sym(h, "MPI_Get_library_version");
        if (rt.ok) {
            static char v[MPI_MAX_LIBRARY_VERSION_STRING];
            int len = 0;
            rt.ok = ver && ver(v, &len) == MPI_SUCCESS &&
                    (strstr(v, "MPICH") || strstr(v, "Intel(R) MPI") || strstr(v, "MVAPICH"));
            if (!rt.ok)
                fprintf(stderr, "libmceik_hip: the loaded MPI is not MPICH-ABI (%.60s); "
                                "the MPI entry points run as a single process\n", ver ? v : "no MPI_Get_library_version");
        }
    }
    if (!rt.ok) return 0;
    int a = 0, b = 0;
    return rt.initialized(&a) == MPI_SUCCESS && a && rt.finalized(&b) == MPI_SUCCESS && !b;
}

/* Rank of the caller in the Fortran communicator handle fcomm, or -1 when
 * this process runs no (initialised) MPI or the handle is not a communicator. */
MCEIK_HIDDEN int mceik_mpi_rank(int fcomm)
{
    if (!load()) return -1;
    int r = -1;
    return rt.rank(MPI_Comm_f2c((MPI_Fint)fcomm), &r) == MPI_SUCCESS ? r : -1;
}

MCEIK_HIDDEN int mceik_mpi_bcast_int(int fcomm, int *v, int n, int root)
{
    if (!load()) return -1;
    return rt.bcast(v, n, MPI_INT, root, MPI_Comm_f2c((MPI_Fint)fcomm)) == MPI_SUCCESS ? 0 : -1;
}

MCEIK_HIDDEN int mceik_mpi_bcast_double(int fcomm, double *v, int n, int root)
{
    if (!load()) return -1;
    return rt.bcast(v, n, MPI_DOUBLE, root, MPI_Comm_f2c((MPI_Fint)fcomm)) == MPI_SUCCESS ? 0 : -1;
}

/* The block-decomposed solve across ranks (fsm3d.f90:103-222 with
 * EIKONAL_EXCHANGE :971-1046 and the gather of EIKONAL_GATHER_TRAVELTIMES):
 * communicator size, an integer all-reduce (op 0 sum, 1 max), an all-gather of
 * fixed-size byte records, and a batch of non-blocking double sends/receives
 * completed together (the halo swap: every rank posts all of its faces, so no
 * ordering can deadlock). */
MCEIK_HIDDEN int mceik_mpi_size(int fcomm)
{
    if (!load()) return -1;
    int n = -1;
    return rt.size(MPI_Comm_f2c((MPI_Fint)fcomm), &n) == MPI_SUCCESS ? n : -1;
}

MCEIK_HIDDEN int mceik_mpi_allreduce_int(int fcomm, int *v, int n, int op)
{
    if (!load()) return -1;
    return rt.allreduce(MPI_IN_PLACE, v, n, MPI_INT, op ? MPI_MAX : MPI_SUM, MPI_Comm_f2c((MPI_Fint)fcomm)) ==
                   MPI_SUCCESS ? 0 : -1;
}

MCEIK_HIDDEN int mceik_mpi_allgather_bytes(int fcomm, const void *mine, void *all, int nbytes)
{
    if (!load()) return -1;
    return rt.allgather(mine, nbytes, MPI_BYTE, all, nbytes, MPI_BYTE, MPI_Comm_f2c((MPI_Fint)fcomm)) ==
                   MPI_SUCCESS ? 0 : -1;
}

/* Fixed-size byte records: root receives every rank's `mine` into `all`
 * (rank order) / sends record r of `all` to rank r; a byte broadcast; a
 * barrier (the h5io and broadcast entry points, csrc/h5io_mpi.c, broadcast.c). */
MCEIK_HIDDEN int mceik_mpi_gather_bytes(int fcomm, const void *mine, void *all, long long nbytes, int root)
{
    if (!load() || nbytes < 0 || nbytes > 0x7fffffffLL) return -1;
    return rt.gather(mine, (int)nbytes, MPI_BYTE, all, (int)nbytes, MPI_BYTE, root, MPI_Comm_f2c((MPI_Fint)fcomm)) ==
                   MPI_SUCCESS ? 0 : -1;
}

MCEIK_HIDDEN int mceik_mpi_scatter_bytes(int fcomm, const void *all, void *mine, long long nbytes, int root)
{
    if (!load() || nbytes < 0 || nbytes > 0x7fffffffLL) return -1;
    return rt.scatter(all, (int)nbytes, MPI_BYTE, mine, (int)nbytes, MPI_BYTE, root, MPI_Comm_f2c((MPI_Fint)fcomm)) ==
                   MPI_SUCCESS ? 0 : -1;
}

MCEIK_HIDDEN int mceik_mpi_bcast_bytes(int fcomm, void *v, long long nbytes, int root)
{
    if (!load() || nbytes < 0 || nbytes > 0x7fffffffLL) return -1;
    return rt.bcast(v, (int)nbytes, MPI_BYTE, root, MPI_Comm_f2c((MPI_Fint)fcomm)) == MPI_SUCCESS ? 0 : -1;
}

MCEIK_HIDDEN int mceik_mpi_barrier(int fcomm)
{
    if (!load()) return -1;
    return rt.barrier(MPI_Comm_f2c((MPI_Fint)fcomm)) == MPI_SUCCESS ? 0 : -1;
}

/* Communicator construction for mpiutils.c (Fortran handles in and out):
 * a duplicate, a split by colour (key = rank), and a free. */
MCEIK_HIDDEN int mceik_mpi_comm_dup(int fcomm, int *fout)
{
    if (!load()) return -1;
    MPI_Comm c;
    if (rt.dup(MPI_Comm_f2c((MPI_Fint)fcomm), &c) != MPI_SUCCESS) return -1;
    *fout = (int)MPI_Comm_c2f(c);
    return 0;
}

MCEIK_HIDDEN int mceik_mpi_comm_split(int fcomm, int color, int key, int *fout)
{
    if (!load()) return -1;
    MPI_Comm c;
    if (rt.split(MPI_Comm_f2c((MPI_Fint)fcomm), color, key, &c) != MPI_SUCCESS) return -1;
    *fout = (int)MPI_Comm_c2f(c);
    return 0;
}

MCEIK_HIDDEN int mceik_mpi_comm_free(int fcomm)
{
    if (!load()) return -1;
    MPI_Comm c = MPI_Comm_f2c((MPI_Fint)fcomm);
    return rt.cfree(&c) == MPI_SUCCESS ? 0 : -1;
}

/* nmsg messages: send[k] (count[k] doubles to peer[k], tag tag[k]) when
 * dir[k] = 0, receive (from peer[k]) when dir[k] = 1; all complete on return. */
MCEIK_HIDDEN int mceik_mpi_exchange_double(int fcomm, int nmsg, const int *dir, const int *peer, const int *tag,
                                           double *const *buf, const int *count)
{
    if (!load()) return -1;
    if (nmsg <= 0) return 0;
    MPI_Comm c = MPI_Comm_f2c((MPI_Fint)fcomm);
    MPI_Request rq[64], *req = nmsg <= 64 ? rq : (MPI_Request *)malloc(sizeof(MPI_Request) * (size_t)nmsg);
    if (!req) return -1;
    int bad = 0;
    for (int k = 0; k < nmsg; k++) {
        const int r = dir[k] ? rt.irecv(buf[k], count[k], MPI_DOUBLE, peer[k], tag[k], c, &req[k])
                             : rt.isend(buf[k], count[k], MPI_DOUBLE, peer[k], tag[k], c, &req[k]);
        if (r != MPI_SUCCESS) { req[k] = MPI_REQUEST_NULL; bad = 1; }
    }
    if (rt.waitall(nmsg, req, MPI_STATUSES_IGNORE) != MPI_SUCCESS) bad = 1;
    if (req != rq) free(req);
    return bad ? -1 : 0;
}
#else
MCEIK_HIDDEN int mceik_mpi_rank(int fcomm) { (void)fcomm; return -1; }
MCEIK_HIDDEN int mceik_mpi_bcast_int(int fcomm, int *v, int n, int root)
{
    (void)fcomm; (void)v; (void)n; (void)root;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_bcast_double(int fcomm, double *v, int n, int root)
{
    (void)fcomm; (void)v; (void)n; (void)root;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_size(int fcomm) { (void)fcomm; return -1; }
MCEIK_HIDDEN int mceik_mpi_allreduce_int(int fcomm, int *v, int n, int op)
{
    (void)fcomm; (void)v; (void)n; (void)op;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_allgather_bytes(int fcomm, const void *mine, void *all, int nbytes)
{
    (void)fcomm; (void)mine; (void)all; (void)nbytes;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_exchange_double(int fcomm, int nmsg, const int *dir, const int *peer, const int *tag,
                                           double *const *buf, const int *count)
{
    (void)fcomm; (void)nmsg; (void)dir; (void)peer; (void)tag; (void)buf; (void)count;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_gather_bytes(int fcomm, const void *mine, void *all, long long nbytes, int root)
{
    (void)fcomm; (void)mine; (void)all; (void)nbytes; (void)root;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_scatter_bytes(int fcomm, const void *all, void *mine, long long nbytes, int root)
{
    (void)fcomm; (void)all; (void)mine; (void)nbytes; (void)root;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_bcast_bytes(int fcomm, void *v, long long nbytes, int root)
{
    (void)fcomm; (void)v; (void)nbytes; (void)root;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_barrier(int fcomm) { (void)fcomm; return -1; }
MCEIK_HIDDEN int mceik_mpi_comm_dup(int fcomm, int *fout) { (void)fcomm; (void)fout; return -1; }
MCEIK_HIDDEN int mceik_mpi_comm_split(int fcomm, int color, int key, int *fout)
{
    (void)fcomm; (void)color; (void)key; (void)fout;
    return -1;
}
MCEIK_HIDDEN int mceik_mpi_comm_free(int fcomm) { (void)fcomm; return -1; }
#endif
