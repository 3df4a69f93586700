// fsm_single.h -- host/device description of one whole-GPU eikonal solve
// (fsm_single.hip).  Not a public header.
#pragma once
#include <stddef.h>
#include <hip/hip_runtime.h>

// Fields are x-fastest on a grid padded to whole 8x8x8 bricks (nxp = 8*nbx ...):
// every brick row is 8 contiguous, aligned values.
struct SingleLaunch {
    int nx, ny, nz, nxp, nyp, nzp;
    int nbx, nby, nbz, nb;           // bricks
    int maxit;
    double tol, h, x0, y0, z0;
    void *u, *u0;                    // R [nzp][nyp][nxp]
    const void *slow;                // R [nzp][nyp][nxp] (s/m)
    unsigned char *bc;               // [nzp][nyp][nxp] 1 = boundary-condition node (lupd = .FALSE.)
    const int *border;               // [nb] bricks in sweep coordinates bx | by << 10 | bz << 20, by level
    unsigned *done;                  // [nb] sweeps completed by each brick
    unsigned *ctl;                   // [0] task counter; [32 + it] iteration it: 0 pending, 1 go on, 2 converged
    unsigned long long *arrive;      // [maxit] bricks done with the iteration | not-converged count << 32
    int *ierr_it;                    // [maxit] ierr of node (0,0,0) in the iteration's last sweep
    const int *bcerr;                // SETBCS failed (ierr = 1): no sweep runs
};

int fsm_single_occupancy(int is_double);
hipError_t fsm_single_solve(const SingleLaunch &L, int is_double, const double *d_src, int nsrc, int *d_ierr_bc,
                            int nwaves, hipStream_t st);
hipError_t fsm_single_pad(const double *src, void *dst, int is_double, int nx, int ny, int nz, int nxp, int nyp,
                          hipStream_t st);
hipError_t fsm_single_unpad(const void *src, double *dst, int is_double, int nx, int ny, int nz, int nxp, int nyp,
                            hipStream_t st);
