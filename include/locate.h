/*
 * locate.h -- the reference's MPI location driver (reference
 * include/locate.h:10-23, locate.f90:322-689), implemented in
 * libmceik_hip.so over the GPU relocation grid search (mceik_relocate), so
 * homog.c:429-450's location step links unchanged.
 *
 * Same names, arguments (Fortran-style pointers, communicator as a Fortran
 * handle, HDF5 file ids as long) and call order (initialize, gridsearch per
 * model, finalize).  The reference's locate.f90 does not compile (SURVEY
 * s.0.5), so the weighting is locate.c's (SURVEY s.8a row a12): weight 1/var,
 * the analytic origin time of Moser eq. 19 (job 2) or the catalogue's tori
 * (job 1), objective = the locate_l2_gridSearch__float64 L2 misfit at every
 * node of the rank's location block; the hypocentre is the first node of the
 * largest log-PDF (-objective) over the blocks, in block order (MAXLOC).
 * Tables come from the travel-time file through the library's h5io entry
 * points (libmceik_h5io.so, resolved at run time).  Deviations, all where the
 * reference is undefined or broken: observation i of event e is used when
 * luseObs[e*nobs + i] != 0 (the reference reads luseObs(iobs), i.e. event
 * 1's flags for every event, locate.f90:396,439); every rank returns the
 * hypocentres (the reference fills only the master's); test[e*nobs + i] =
 * t0 + the table value at the hypocentre for used observations (the
 * reference declares test INTENT(OUT) and never writes it).
 */
#ifndef _locate_h__
#define _locate_h__ 1   /* the reference's guard */
#if defined(__has_include)
#if __has_include(<mpi.h>)
#include <mpi.h>
#endif
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* locate.f90:562-677: comm = the intra-table communicator (homog.c:429);
 * splits it with mpiutils_initialize3d when the harness has not; reads the
 * model dimensions (master) and this rank's block of /Model/{x,y,z}locs. */
void locate3d_initialize(const int *comm, const int *iverb,
                         const long *tttFileID, const long *locFileID,
                         const int *ndivx, const int *ndivy, const int *ndivz,
                         int *ierr);

/* locate.f90:322-519: job 1 location only (t0 = tori), 2 location and
 * origin time; 3 and 5 are "not yet done" there (ierr 1), as here.
 * Arrays are [nevents*nobs] (statPtr 1-based stations, pickType 1 P /
 * 2 S), statCor [nobs], tori [nevents], hypo [4*nevents] = x, y, z, t0. */
void locate3d_gridsearch(const int *model,
                         const int *job, const int *nobs, const int *nevents,
                         const int *luseObs, const int *statPtr,
                         const int *pickType, const double *statCor,
                         const double *tori, const double *varobs,
                         const double *tobs, double *test,
                         double *hypo, int *ierr);

/* locate.f90:681-689 */
void locate3d_finalize(void);

#ifdef __cplusplus
}
#endif
#endif /* _locate_h__ */
