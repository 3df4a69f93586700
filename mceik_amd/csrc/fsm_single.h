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
    // The fields may hold a box of a larger grid (the MPI variant across ranks:
    // a rank's block and its ghost layer): global dimensions and the global
    // coordinates of local node 0.  The whole grid: g = n, o = 0.
    int gx, gy, gz, ox, oy, oz;
};

// Block decomposition of the MPI variant (fsm3d.f90:1086-1101): nd blocks per
// axis, block b owning [step*b, step*(b+1)-1] (the last one up to n-1), ghost
// layer width nov (0: block faces are grid edges).
struct BlockDecomp {
    int nd[3], step[3], nov;
};

// A box of grid nodes [lo, lo + ext) and a list of them packed back to back
// (box k at off[k] doubles; off[n] = total).
struct BlockBox {
    int lo[3], ext[3];
};
struct BoxList {
    int n;
    BlockBox box[6];
    size_t off[7];
};

int fsm_single_occupancy(int is_double);
hipError_t fsm_single_setbcs(const SingleLaunch &L, const double *d_src, int nsrc, int *d_ierr_bc, hipStream_t st);
// nblk blocks from b0 (nblk < 0: every block); ierr_b: the block whose
// last-level ierr is reported
hipError_t fsm_block_sweep(const SingleLaunch &L, const BlockDecomp &D, const double *snap, int g, int *ierr,
                           hipStream_t st, int b0 = 0, int nblk = -1, int ierr_b = 0);
hipError_t fsm_block_unconverged(const SingleLaunch &L, const BlockBox &B, double tol, unsigned *count,
                                 hipStream_t st);
hipError_t fsm_box_copy(const SingleLaunch &L, const BoxList &bl, double *buf, int to_buf, hipStream_t st);
hipError_t fsm_single_solve(const SingleLaunch &L, int is_double, const double *d_src, int nsrc, int *d_ierr_bc,
                            int nwaves, hipStream_t st);
hipError_t fsm_single_pad(const double *src, void *dst, int is_double, int nx, int ny, int nz, int nxp, int nyp,
                          hipStream_t st);
hipError_t fsm_single_unpad(const void *src, double *dst, int is_double, int nx, int ny, int nz, int nxp, int nyp,
                            hipStream_t st);
