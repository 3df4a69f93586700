/* h5io.c -- posterior / travel-time HDF5 files in the reference's layout.
 *
 * Serial (rank 0 after the RCCL gather, SURVEY s.8f row 1) restatement of the
 * reference's h5io.c layout:
 *   <dir>/<proj>_ttimes.h5     (h5io.c:50-57, initTTables :559-712)
 *     /Model/{xlocs,ylocs,zlocs}                 fp32, dataspace {nx,ny,nz}
 *     /TravelTimeTables/Model_m/Station_s/{P,S}TravelTimes     (h5io.c:164-181)
 *   <dir>/<proj>_locations.h5  (initLocations :232-416)
 *     /Model/{xlocs,ylocs,zlocs}, /Model/priorLocationModel (= 1.0)
 *     /logJPDFs/Event_e/Model_m/logJPDF                        (h5io.c:183-190)
 * Layout quirk kept on purpose (h5io.c:254,433,464,760,900): the file
 * dataspace is {nx, ny, nz} (C order, z fastest in the file) but it is filled
 * straight from an x-fastest buffer, so a reader must reinterpret the raw
 * data as [nz][ny][nx].  Models and stations are 1-based as in the reference.
 * The reference uses parallel HDF5 with per-rank hyperslabs; here one process
 * writes whole grids (ix0 = iy0 = iz0 = 0, nxLoc = nx ...).
 */
#include <limits.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <hdf5.h>

#include "../../include/mceik_h5io.h"

int eikonal_h5io_setFileName(int job, const char *dirnm, const char *projnm, char fileName[PATH_MAX])
{
    const char *fcnm = "eikonal_h5io_setFileName";
    memset(fileName, 0, PATH_MAX);
    if (dirnm == NULL || strlen(dirnm) == 0) {
        strcpy(fileName, "./");
    } else {
        if (strlen(dirnm) + 2 >= PATH_MAX) return -1;
        strcpy(fileName, dirnm);
        if (fileName[strlen(fileName) - 1] != '/') strcat(fileName, "/");
    }
    if (projnm == NULL) {
        printf("%s: Project name must be defined\n", fcnm);
        return -1;
    }
    if (strlen(projnm) == 0) {
        printf("%s: Project can't be empty\n", fcnm);
        return -1;
    }
    if (strlen(fileName) + strlen(projnm) + 16 >= PATH_MAX) return -1;
    strcat(fileName, projnm);
    if (job == MCEIK_H5_TRAVELTIME_FILE) strcat(fileName, "_ttimes.h5");
    else if (job == MCEIK_H5_LOCATION_FILE) strcat(fileName, "_locations.h5");
    return 0;
}

void eikonal_h5io_setTravelTimeName(int model, int station, bool isP, char dataSetName[512])
{
    memset(dataSetName, 0, 512);
    snprintf(dataSetName, 512, "/TravelTimeTables/Model_%d/Station_%d/%sTravelTimes", model, station,
             isP ? "P" : "S");
}

void eikonal_h5io_setLocationName(int model, int event, char dataSetName[512])
{
    memset(dataSetName, 0, 512);
    snprintf(dataSetName, 512, "/logJPDFs/Event_%d/Model_%d/logJPDF", event, model);
}

static int make_group(hid_t fid, const char *name)
{
    hid_t g = H5Gcreate2(fid, name, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    if (g < 0) return -1;
    return H5Gclose(g) < 0 ? -1 : 0;
}

/* fp32 dataset with dataspace {nx, ny, nz}; data (may be NULL: created only,
 * reads back as the fill value 0, like the reference's null writes) is the
 * x-fastest buffer written as-is (the layout quirk). */
static int write_grid(hid_t fid, const char *name, int nx, int ny, int nz, const float *data, int create)
{
    const hsize_t dims[3] = {(hsize_t)nx, (hsize_t)ny, (hsize_t)nz};
    hid_t ds;
    if (create) {
        hid_t sp = H5Screate_simple(3, dims, NULL);
        if (sp < 0) return -1;
        ds = H5Dcreate2(fid, name, H5T_NATIVE_FLOAT, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
        H5Sclose(sp);
    } else {
        if (H5Lexists(fid, name, H5P_DEFAULT) <= 0) {
            printf("mceik_h5io: dataset %s doesn't exist\n", name);
            return -1;
        }
        ds = H5Dopen2(fid, name, H5P_DEFAULT);
    }
    if (ds < 0) return -1;
    int rc = 0;
    if (data && H5Dwrite(ds, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0) rc = -1;
    if (H5Dclose(ds) < 0) rc = -1;
    return rc;
}

static int read_grid(hid_t fid, const char *name, int nx, int ny, int nz, float *data)
{
    if (H5Lexists(fid, name, H5P_DEFAULT) <= 0) return -1;
    hid_t ds = H5Dopen2(fid, name, H5P_DEFAULT);
    if (ds < 0) return -1;
    hid_t sp = H5Dget_space(ds);
    hsize_t dims[3] = {0, 0, 0};
    int rc = (H5Sget_simple_extent_ndims(sp) == 3 && H5Sget_simple_extent_dims(sp, dims, NULL) == 3 &&
              dims[0] == (hsize_t)nx && dims[1] == (hsize_t)ny && dims[2] == (hsize_t)nz) ? 0 : -1;
    if (rc == 0 && H5Dread(ds, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0) rc = -1;
    H5Sclose(sp);
    H5Dclose(ds);
    return rc;
}

/* /Model/{x,y,z}locs (h5io.c:418-534): (float)(x0 + i*dx) etc., x fastest. */
static int make_model_group(hid_t fid, int nx, int ny, int nz, double x0, double y0, double z0, double dx,
                            double dy, double dz)
{
    if (make_group(fid, "/Model") != 0) return -1;
    const size_t n = (size_t)nx * ny * nz;
    float *buf = (float *)malloc(n * sizeof(float));
    if (!buf) return -1;
    static const char *names[3] = {"/Model/xlocs", "/Model/ylocs", "/Model/zlocs"};
    int rc = 0;
    for (int v = 0; v < 3 && rc == 0; v++) {
        for (int k = 0; k < nz; k++)
            for (int j = 0; j < ny; j++)
                for (int i = 0; i < nx; i++) {
                    const size_t idx = ((size_t)k * ny + j) * nx + i;
                    buf[idx] = v == 0 ? (float)(x0 + (double)i * dx)
                             : v == 1 ? (float)(y0 + (double)j * dy) : (float)(z0 + (double)k * dz);
                }
        rc = write_grid(fid, names[v], nx, ny, nz, buf, 1);
    }
    free(buf);
    return rc;
}

int mceik_h5io_initTTables(const char *dirnm, const char *projnm, int nx, int ny, int nz, int nmodels,
                           int nstations, double x0, double y0, double z0, double dx, double dy, double dz,
                           int64_t *fileID)
{
    char h5name[PATH_MAX], name[512];
    if (!fileID || nx < 1 || ny < 1 || nz < 1 || nmodels < 0 || nstations < 0) return -1;
    if (eikonal_h5io_setFileName(MCEIK_H5_TRAVELTIME_FILE, dirnm, projnm, h5name) != 0) return -1;
    hid_t fid = H5Fcreate(h5name, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    if (fid < 0) {
        printf("mceik_h5io_initTTables: cannot create %s\n", h5name);
        return -1;
    }
    int rc = make_model_group(fid, nx, ny, nz, x0, y0, z0, dx, dy, dz);
    if (rc == 0) rc = make_group(fid, "/TravelTimeTables");
    for (int m = 1; m <= nmodels && rc == 0; m++) {
        snprintf(name, sizeof(name), "/TravelTimeTables/Model_%d", m);
        rc = make_group(fid, name);
        for (int s = 1; s <= nstations && rc == 0; s++) {
            snprintf(name, sizeof(name), "/TravelTimeTables/Model_%d/Station_%d", m, s);
            rc = make_group(fid, name);
            for (int ph = 0; ph < 2 && rc == 0; ph++) {
                eikonal_h5io_setTravelTimeName(m, s, ph == 0, name);
                rc = write_grid(fid, name, nx, ny, nz, NULL, 1);
            }
        }
    }
    if (rc != 0) {
        H5Fclose(fid);
        return -1;
    }
    *fileID = (int64_t)fid;
    return 0;
}

int mceik_h5io_writeTravelTimes(int64_t fileID, int station, int model, int iphase, int nx, int ny, int nz,
                                const float *ttimes)
{
    char name[512];
    if (!ttimes) return -1;
    eikonal_h5io_setTravelTimeName(model, station, iphase != 2, name);
    return write_grid((hid_t)fileID, name, nx, ny, nz, ttimes, 0);
}

int mceik_h5io_readTravelTimes(int64_t fileID, int station, int model, int iphase, int nx, int ny, int nz,
                               float *ttimes)
{
    char name[512];
    if (!ttimes) return -1;
    eikonal_h5io_setTravelTimeName(model, station, iphase != 2, name);
    return read_grid((hid_t)fileID, name, nx, ny, nz, ttimes);
}

int mceik_h5io_initLocations(const char *dirnm, const char *projnm, int nx, int ny, int nz, int nmodels,
                             int nevents, double x0, double y0, double z0, double dx, double dy, double dz,
                             int64_t *locFileID)
{
    char h5name[PATH_MAX], name[512];
    if (!locFileID || nx < 1 || ny < 1 || nz < 1 || nmodels < 0 || nevents < 0) return -1;
    if (eikonal_h5io_setFileName(MCEIK_H5_LOCATION_FILE, dirnm, projnm, h5name) != 0) return -1;
    hid_t fid = H5Fcreate(h5name, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    if (fid < 0) {
        printf("mceik_h5io_initLocations: cannot create %s\n", h5name);
        return -1;
    }
    int rc = make_model_group(fid, nx, ny, nz, x0, y0, z0, dx, dy, dz);
    if (rc == 0) {                                   // uniform prior (h5io.c:308-343)
        const size_t n = (size_t)nx * ny * nz;
        float *one = (float *)malloc(n * sizeof(float));
        if (!one) rc = -1;
        for (size_t i = 0; one && i < n; i++) one[i] = 1.0f;
        if (rc == 0) rc = write_grid(fid, "/Model/priorLocationModel", nx, ny, nz, one, 1);
        free(one);
    }
    if (rc == 0) rc = make_group(fid, "/logJPDFs");
    for (int e = 1; e <= nevents && rc == 0; e++) {
        snprintf(name, sizeof(name), "/logJPDFs/Event_%d", e);
        rc = make_group(fid, name);
        for (int m = 1; m <= nmodels && rc == 0; m++) {
            snprintf(name, sizeof(name), "/logJPDFs/Event_%d/Model_%d", e, m);
            rc = make_group(fid, name);
            eikonal_h5io_setLocationName(m, e, name);
            if (rc == 0) rc = write_grid(fid, name, nx, ny, nz, NULL, 1);
        }
    }
    if (rc != 0) {
        H5Fclose(fid);
        return -1;
    }
    *locFileID = (int64_t)fid;
    return 0;
}

int mceik_h5io_writeLocationLogJPDF(int64_t locFileID, int model, int event, int nx, int ny, int nz,
                                    const float *logJPDF)
{
    char name[512];
    if (!logJPDF) return -1;
    eikonal_h5io_setLocationName(model, event, name);
    return write_grid((hid_t)locFileID, name, nx, ny, nz, logJPDF, 0);
}

int mceik_h5io_readLocationLogJPDF(int64_t locFileID, int model, int event, int nx, int ny, int nz,
                                   float *logJPDF)
{
    char name[512];
    if (!logJPDF) return -1;
    eikonal_h5io_setLocationName(model, event, name);
    return read_grid((hid_t)locFileID, name, nx, ny, nz, logJPDF);
}

int mceik_h5io_getModelDimensions(int64_t fileID, int *nx, int *ny, int *nz)
{
    if (!nx || !ny || !nz) return -1;
    hid_t fid = (hid_t)fileID;
    if (H5Lexists(fid, "/Model/xlocs", H5P_DEFAULT) <= 0) return -1;
    hid_t ds = H5Dopen2(fid, "/Model/xlocs", H5P_DEFAULT);
    hid_t sp = H5Dget_space(ds);
    hsize_t dims[3] = {0, 0, 0};
    int rc = H5Sget_simple_extent_ndims(sp) == 3 && H5Sget_simple_extent_dims(sp, dims, NULL) == 3 ? 0 : -1;
    H5Sclose(sp);
    H5Dclose(ds);
    if (rc == 0) {                                   // dataspace {nx, ny, nz} (the quirk)
        *nx = (int)dims[0]; *ny = (int)dims[1]; *nz = (int)dims[2];
    }
    return rc;
}

int mceik_h5io_readModel(int64_t fileID, int nx, int ny, int nz, float *xlocs, float *ylocs, float *zlocs)
{
    hid_t fid = (hid_t)fileID;
    if (xlocs && read_grid(fid, "/Model/xlocs", nx, ny, nz, xlocs) != 0) return -1;
    if (ylocs && read_grid(fid, "/Model/ylocs", nx, ny, nz, ylocs) != 0) return -1;
    if (zlocs && read_grid(fid, "/Model/zlocs", nx, ny, nz, zlocs) != 0) return -1;
    return 0;
}

int mceik_h5io_exists(int64_t fileID, const char *name)
{
    return name && H5Lexists((hid_t)fileID, name, H5P_DEFAULT) > 0 ? 1 : 0;
}

int mceik_h5io_open(const char *fileName, int readwrite, int64_t *fileID)
{
    if (!fileName || !fileID) return -1;
    hid_t fid = H5Fopen(fileName, readwrite ? H5F_ACC_RDWR : H5F_ACC_RDONLY, H5P_DEFAULT);
    if (fid < 0) return -1;
    *fileID = (int64_t)fid;
    return 0;
}

int mceik_h5io_finalize(int64_t *fileID)
{
    if (!fileID) return -1;
    if (H5Fclose((hid_t)*fileID) < 0) {
        printf("mceik_h5io_finalize: Failed closing file\n");
        return -1;
    }
    *fileID = -1;
    return 0;
}
