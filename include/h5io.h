/*
 * h5io.h -- the reference's travel-time / location HDF5 interface
 * (reference include/h5io.h:18-106, h5io.c), drop-in for a homog.c-style MPI
 * harness: same names, argument meaning, 1-based model / station / event
 * numbers, file and dataset layout, and return codes (0 = success).
 *
 * The reference writes with parallel HDF5 (every rank its hyperslab of the
 * {nx, ny, nz} dataspace, collective MPI-IO).  The image's HDF5 is serial, so
 * libmceik_h5io.so keeps the reference's arguments but moves the data: rank 0
 * of `comm` owns the file; every rank's block (its nxLoc x nyLoc x nzLoc
 * buffer zero-padded to the communicator's max block, as the reference packs
 * it, h5io.c:893-905) travels to rank 0, which writes each rank's hyperslab
 * {ix0, iy0, iz0} + {nxMax, nyMax, nzMax} in rank order with the same
 * H5Dwrite the reference issues (memory space {nxMax, nyMax, nzMax} over the
 * x-fastest buffer: the file holds what the reference's collective write
 * leaves; where blocks overlap, the higher rank's write lands last).  Reads
 * are the inverse (rank 0 reads each rank's hyperslab and scatters).  Every
 * rank returns the same code.  A process without (initialised) MPI is rank 0
 * of one.  Ranks other than 0 hold a handle that only this library knows
 * (getModelDimensions answers from it).  MPI is resolved at run time from the
 * caller's MPICH-ABI MPI (csrc/mpi_rt.c), as in libmceik_hip.so.
 */
#include <stdbool.h>
#include <limits.h>
#include <hdf5.h>
#include <mpi.h>
#ifndef _h5io_h__
#define _h5io_h__ 1
#ifdef __cplusplus
extern "C" {
#endif

enum fileName_enum { TRAVELTIME_FILE = 1, LOCATION_FILE = 2 };
/* h5io.c:192-204: closes the file (rank 0) / releases the handle (others). */
int eikonal_h5io_finalize(const MPI_Comm comm, hid_t *tttFileID);
/* h5io.c:9-58: "<dirnm>/<projnm>_ttimes.h5" (job 1) or "_locations.h5" (job 2). */
int eikonal_h5io_setFileName(enum fileName_enum job, const char *dirnm, const char *projnm,
                             char fileName[PATH_MAX]);
/* h5io.c:164-181: /TravelTimeTables/Model_<m>/Station_<s>/{P,S}TravelTimes */
void eikonal_h5io_setTravelTimeName(const int model, const int station, const bool isP,
                                    char dataSetName[512]);
/* h5io.c:183-190: /logJPDFs/Event_<e>/Model_<m>/logJPDF */
void eikonal_h5io_setLocationName(const int model, const int event, char dataSetName[512]);
/* h5io.c:76-162: dims of /Model/xlocs (rank 1: nx = ny = nz = dims[0]). */
void eikonal_h5io_getModelDimensionsF(const long *inFileID, int *nx, int *ny, int *nz, int *ierr);
int eikonal_h5io_getModelDimensions(const hid_t fileID, int *nx, int *ny, int *nz);
/* h5io.c:960-1156: this rank's block of /Model/{x,y,z}locs (F: 1-based offsets). */
void eikonal_h5io_readModelF(const int *comm, const long *inFileID, const int *ix0, const int *iy0,
                             const int *iz0, const int *nxLoc, const int *nyLoc, const int *nzLoc,
                             float *__restrict__ xlocs, float *__restrict__ ylocs, float *__restrict__ zlocs,
                             int *ierr);
int eikonal_h5io_readModel(const MPI_Comm comm, const hid_t fileID, const int ix0, const int iy0,
                           const int iz0, const int nxLoc, const int nyLoc, const int nzLoc,
                           float *__restrict__ xlocs, float *__restrict__ ylocs, float *__restrict__ zlocs);
/* h5io.c:232-416: model group, uniform /Model/priorLocationModel, zero
 * /logJPDFs/Event_e/Model_m/logJPDF for every event and model. */
int eikonal_h5io_initLocations(const MPI_Comm comm, const char *dirnm, const char *projnm, const int ix0,
                               const int iy0, const int iz0, const int nx, const int ny, const int nz,
                               const int nxLoc, const int nyLoc, const int nzLoc, const int nmodels,
                               const int nevents, const double x0, const double y0, const double z0,
                               const double dx, const double dy, const double dz, hid_t *locFileID);
/* h5io.c:559-712: model group and zero {P,S}TravelTimes of every model and
 * station (lsaveScratch: the reference's in-RAM option, unsupported there too). */
int eikonal_h5io_initTTables(const MPI_Comm comm, const char *dirnm, const char *projnm, const int ix0,
                             const int iy0, const int iz0, const int nx, const int ny, const int nz,
                             const int nxLoc, const int nyLoc, const int nzLoc, const int nmodels,
                             const int nstations, const bool lsaveScratch, const double x0, const double y0,
                             const double z0, const double dx, const double dy, const double dz,
                             hid_t *tttFileID);
/* h5io.c:418-534 */
int eikonal_h5io_makeModelGroup(const MPI_Comm comm, const hid_t fileID, const int ix0, const int iy0,
                                const int iz0, const int nxGlob, const int nyGlob, const int nzGlob,
                                const int nxLoc, const int nyLoc, const int nzLoc, const int nxMax,
                                const int nyMax, const int nzMax, const double dx, const double dy,
                                const double dz, const double x0, const double y0, const double z0);
/* h5io.c:1226-1341 (F: h5io.c:1162-1193, 1-based offsets, ttimes zeroed on error) */
int eikonal_h5io_readTravelTimes(const MPI_Comm comm, const hid_t tttFileID, const int station,
                                 const int model, const int iphase, const int ix0, const int iy0,
                                 const int iz0, const int nxLoc, const int nyLoc, const int nzLoc,
                                 float *__restrict__ ttimes);
void eikonal_h5io_readTraveltimesF(const int *comm, const long *tttFileID, const int *station,
                                   const int *model, const int *iphase, const int *ix0f, const int *iy0f,
                                   const int *iz0f, const int *nxLoc, const int *nyLoc, const int *nzLoc,
                                   float *ttimes, int *ierr);
/* h5io.c:851-958: ttimes [nzLoc][nyLoc][nxLoc], x fastest */
int eikonal_h5io_writeTravelTimes(const MPI_Comm comm, const hid_t tttFileID, const int station,
                                  const int model, const int iphase, const int ix0, const int iy0,
                                  const int iz0, const int nxLoc, const int nyLoc, const int nzLoc,
                                  const float *__restrict__ ttimes);
/* h5io.c:714-819 */
int eikonal_h5io_writeLocationLogJPDF(const MPI_Comm comm, const hid_t locFileID, const int model,
                                      const int event, const int ix0, const int iy0, const int iz0,
                                      const int nxLoc, const int nyLoc, const int nzLoc,
                                      const float *__restrict__ logJPDF);

#ifdef __cplusplus
}
#endif
#endif /* _h5io_h__ */
