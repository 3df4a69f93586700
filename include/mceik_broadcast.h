/*
 * mceik_broadcast.h -- station list and catalog from `root` to every rank of
 * `comm` (reference include/mceik_broadcast.h:12-16, broadcast.c:14-143):
 * the same fields in the same order, non-root ranks allocating the arrays
 * (calloc, 64-byte name strings) that the caller frees as homog.c's
 * freeStations / freeCatalog do.  Implemented in libmceik_hip.so over the
 * caller's MPI, resolved at run time (csrc/mpi_rt.c); a process without
 * (initialised) MPI is a single rank and keeps its data.
 */
#ifndef _mceik_broadcast_h__
#define _mceik_broadcast_h__ 1
#include <mpi.h>
#include "mceik_struct.h"
#ifdef __cplusplus
extern "C" {
#endif
void broadcast_catalog(MPI_Comm comm, const int root, struct mceik_catalog_struct *catalog);
void broadcast_stations(MPI_Comm comm, const int root, struct mceik_stations_struct *stations);
#ifdef __cplusplus
}
#endif
#endif
