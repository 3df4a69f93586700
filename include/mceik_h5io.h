/*
 * mceik_h5io.h -- posterior / travel-time HDF5 files (libmceik_h5io.so).
 *
 * The reference's h5io layout (h5io.c:9-1341, h5io.h) written serially by
 * one process (rank 0 after the RCCL gather of kept samples; SURVEY s.8f
 * row 1).  File names, group/dataset names, fp32 datasets, 1-based model /
 * station / event numbers and the {nx,ny,nz}-dataspace-over-x-fastest-data
 * quirk are the reference's; the MPI communicator and per-rank hyperslab
 * arguments are dropped because one process writes whole grids.
 * File handles are HDF5 hid_t values (int64_t in HDF5 >= 1.10).
 */
#ifndef MCEIK_H5IO_H_AMD
#define MCEIK_H5IO_H_AMD 1
#include <limits.h>
#include <stdbool.h>
#include <stdint.h>
#ifndef PATH_MAX
#define PATH_MAX 4096
#endif

#ifdef __cplusplus
extern "C" {
#endif

enum { MCEIK_H5_TRAVELTIME_FILE = 1, MCEIK_H5_LOCATION_FILE = 2 };   /* h5io.h:12-16 */

/* h5io.c:9-58: "<dir>/<proj>_ttimes.h5" (job 1) or "_locations.h5" (job 2). */
int eikonal_h5io_setFileName(int job, const char *dirnm, const char *projnm, char fileName[PATH_MAX]);
/* h5io.c:164-181 / 183-190 */
void eikonal_h5io_setTravelTimeName(int model, int station, bool isP, char dataSetName[512]);
void eikonal_h5io_setLocationName(int model, int event, char dataSetName[512]);

/* Replaces eikonal_h5io_initTTables (h5io.c:559-712): /Model/{x,y,z}locs and
 * empty /TravelTimeTables/Model_m/Station_s/{P,S}TravelTimes for m <= nmodels,
 * s <= nstations. */
int mceik_h5io_initTTables(const char *dirnm, const char *projnm, int nx, int ny, int nz, int nmodels,
                           int nstations, double x0, double y0, double z0, double dx, double dy, double dz,
                           int64_t *fileID);
/* Replaces eikonal_h5io_writeTravelTimes / readTravelTimes (h5io.c:851-958,
 * 1226-1341); iphase 1 = P, 2 = S; ttimes [nz][ny][nx] x fastest. */
int mceik_h5io_writeTravelTimes(int64_t fileID, int station, int model, int iphase, int nx, int ny, int nz,
                                const float *ttimes);
int mceik_h5io_readTravelTimes(int64_t fileID, int station, int model, int iphase, int nx, int ny, int nz,
                               float *ttimes);

/* Replaces eikonal_h5io_initLocations (h5io.c:232-416): model group, the
 * uniform /Model/priorLocationModel = 1.0, and empty
 * /logJPDFs/Event_e/Model_m/logJPDF datasets. */
int mceik_h5io_initLocations(const char *dirnm, const char *projnm, int nx, int ny, int nz, int nmodels,
                             int nevents, double x0, double y0, double z0, double dx, double dy, double dz,
                             int64_t *locFileID);
/* Replaces eikonal_h5io_writeLocationLogJPDF (h5io.c:714-806). */
int mceik_h5io_writeLocationLogJPDF(int64_t locFileID, int model, int event, int nx, int ny, int nz,
                                    const float *logJPDF);
int mceik_h5io_readLocationLogJPDF(int64_t locFileID, int model, int event, int nx, int ny, int nz,
                                   float *logJPDF);

/* Replaces eikonal_h5io_getModelDimensions / readModel (h5io.c:107-158,
 * 1018-1160) for a whole grid. */
int mceik_h5io_getModelDimensions(int64_t fileID, int *nx, int *ny, int *nz);
int mceik_h5io_readModel(int64_t fileID, int nx, int ny, int nz, float *xlocs, float *ylocs, float *zlocs);

/* Open an existing file (readwrite != 0: read/write); 1 if `name` exists. */
int mceik_h5io_open(const char *fileName, int readwrite, int64_t *fileID);
int mceik_h5io_exists(int64_t fileID, const char *name);
/* Replaces eikonal_h5io_finalize (h5io.c:192-205). */
int mceik_h5io_finalize(int64_t *fileID);

#ifdef __cplusplus
}
#endif
#endif
