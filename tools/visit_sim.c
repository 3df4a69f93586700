/* visit_sim.c -- analysis tool (not product code): block-level skipping
 * with EXACT information for one fp32 solve.  A z-block (8 x 8 x bz nodes)
 * is updated in a sweep iff it changed at its last visit or a face
 * neighbour changed since then (the batched kernel's rule without its
 * in-flight conservatism and column runs).  Blocks in lexicographic sweep
 * order, nodes lexicographic inside a block: a topological order of the
 * reference's update DAG, so the field is the full sweeps' field.  Reports
 * visited 8x8x8 bricks per sweep against the grid's bricks.
 * build: gcc -O2 -shared -fPIC -o /tmp/visit_sim.so tools/visit_sim.c -lm */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

static float solve3d(float a, float b, float c, float f)
{
    float lo = a < b ? a : b, hi = a < b ? b : a;
    float a1 = lo < c ? lo : c, a3 = hi < c ? c : hi, a2 = lo < c ? (hi < c ? hi : c) : lo;
    if (a1 == FLT_MAX) return FLT_MAX;
    float d2 = a2 - a1, d3 = a3 - a1, y;
    if (!(f > d2)) y = f;
    else {
        float ff = f * f, e = d3 - d2, t = d3 * d3 + e * e;
        if (t >= ff) y = 0.5f * (d2 + sqrtf(ff + ff - d2 * d2));
        else y = (d2 + d3 + sqrtf(3.0f * ff - (d2 * d2 + t))) * (1.0f / 3.0f);
    }
    float x = a1 + y;
    return x < FLT_MAX ? x : FLT_MAX;
}

/* u: initialised field (BCs set), bc: 1 = boundary node; out[0] = iterations,
 * out[1] = visited bricks, out[2] = changed blocks, out[3] = total brick-sweeps */
void visit_sim(int nx, int ny, int nz, int bz, int maxit, float tol, const float *f, const unsigned char *bc,
               float *u, long *out)
{
    const int sw[8][3] = {{0,0,0},{1,0,0},{0,1,0},{1,1,0},{0,0,1},{1,0,1},{0,1,1},{1,1,1}};
    int ntx = (nx + 7) / 8, nty = (ny + 7) / 8, ntz = (nz + bz - 1) / bz;
    long nb = (long)ntx * nty * ntz, n = (long)nx * ny * nz, nxy = (long)nx * ny;
    long *tv = malloc(nb * sizeof(long)), *tc = malloc(nb * sizeof(long));
    float *u0 = malloc(n * sizeof(float));
    for (long b = 0; b < nb; b++) { tv[b] = -2; tc[b] = -3; }
    for (int z = 0; z < nz; z++) for (int y = 0; y < ny; y++) for (int x = 0; x < nx; x++)
        if (bc[z * nxy + (long)y * nx + x]) tc[((long)(z / bz) * nty + y / 8) * ntx + x / 8] = -1;
    long clock = 0, visited = 0, changed_blocks = 0, sweeps_total = 0;
    int it;
    memcpy(u0, u, n * sizeof(float));
    for (it = 1; it <= maxit; it++) {
        for (int s = 0; s < 8; s++) {
            int rx = sw[s][0], ry = sw[s][1], rz = sw[s][2];
            sweeps_total++;
            for (int kbz = 0; kbz < ntz; kbz++) for (int kby = 0; kby < nty; kby++) for (int kbx = 0; kbx < ntx; kbx++) {
                int tbx = rx ? ntx - 1 - kbx : kbx, tby = ry ? nty - 1 - kby : kby, tbz = rz ? ntz - 1 - kbz : kbz;
                long b = ((long)tbz * nty + tby) * ntx + tbx;
                long lp = tv[b];
                int need = tc[b] >= lp;
                if (tbx > 0 && tc[b - 1] > lp) need = 1;
                if (tbx < ntx - 1 && tc[b + 1] > lp) need = 1;
                if (tby > 0 && tc[b - ntx] > lp) need = 1;
                if (tby < nty - 1 && tc[b + ntx] > lp) need = 1;
                if (tbz > 0 && tc[b - (long)ntx * nty] > lp) need = 1;
                if (tbz < ntz - 1 && tc[b + (long)ntx * nty] > lp) need = 1;
                clock++;
                if (!need) continue;
                tv[b] = clock;
                int z0 = tbz * bz, z1 = z0 + bz < nz ? z0 + bz : nz;
                visited += (z1 - z0 + 7) / 8;
                int ch = 0;
                for (int kz = z0; kz < z1; kz++) {
                    int z = rz ? z1 - 1 - (kz - z0) : kz;
                    for (int ky = 0; ky < 8; ky++) {
                        int y = tby * 8 + (ry ? 7 - ky : ky);
                        if (y >= ny) continue;
                        for (int kx = 0; kx < 8; kx++) {
                            int x = tbx * 8 + (rx ? 7 - kx : kx);
                            if (x >= nx) continue;
                            long i = (long)z * nxy + (long)y * nx + x;
                            if (bc[i]) continue;
                            float self = u[i];
                            float xm = x > 0 ? u[i - 1] : self, xp = x < nx - 1 ? u[i + 1] : self;
                            float ym = y > 0 ? u[i - nx] : self, yp = y < ny - 1 ? u[i + nx] : self;
                            float zm = z > 0 ? u[i - nxy] : self, zp = z < nz - 1 ? u[i + nxy] : self;
                            float v = solve3d(xm < xp ? xm : xp, ym < yp ? ym : yp, zm < zp ? zm : zp, f[i]);
                            if (v < self) { u[i] = v; ch = 1; }
                        }
                    }
                }
                if (ch) { tc[b] = clock; changed_blocks++; }
            }
        }
        long conv = 0;
        for (long i = 0; i < n; i++) { if (fabsf(u0[i] - u[i]) < tol) conv++; u0[i] = u[i]; }
        if (conv == n) break;
    }
    out[0] = it > maxit ? maxit : it;
    out[1] = visited;
    out[2] = changed_blocks;
    out[3] = sweeps_total * (long)ntx * nty * ((nz + 7) / 8);
    free(tv); free(tc); free(u0);
}
