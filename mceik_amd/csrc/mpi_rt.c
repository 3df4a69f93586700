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

#define MCEIK_HIDDEN __attribute__((visibility("hidden")))

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

static struct {
    int tried, ok;
    flag_fn initialized, finalized;
    rank_fn rank;
    bcast_fn bcast;
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
        rt.bcast = (bcast_fn)sym(h, "MPI_Bcast");
        rt.ok = rt.initialized && rt.finalized && rt.rank && rt.bcast;
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
#endif
