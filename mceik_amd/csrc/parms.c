/*
 * parms.c -- configuration of a sampler run: mceik_parms_struct + mceik_mcmc_opts
 * from an INI file and "section:key=value" overrides (include/mceik.h).
 *
 * The reference parses nothing: its mains hard-code every parameter
 * (homog.c:73-89, fsm3d.f90:2085-2100) and link iniparser without including
 * it (Makefile.inc:25-26,39).  mceik_parms_struct (mceik_struct.h:68-90) is
 * the intended config record (SURVEY s.5); this file fills it the way an
 * iniparser-based main would: [section] headers, "key = value" lines,
 * ';' or '#' comments, case-insensitive section and key names, optional
 * double quotes around a value, and command-line overrides spelled
 * "section:key=value" (iniparser's own "section:key" addressing).
 *
 * Host-only C (no HIP calls): usable before any device is touched.
 */
#include <ctype.h>
#include <errno.h>
#include <limits.h>
#include <math.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mceik.h"

enum kind { K_INT, K_U32, K_DBL, K_STR };

struct key {
    const char *section, *name;
    enum kind kind;
    int in_opts;          /* 0: offset into mceik_parms_struct, 1: into mceik_mcmc_opts */
    size_t off, cap;      /* cap: K_STR buffer size */
};

#define P(sec, nm, k, member) {sec, nm, k, 0, offsetof(struct mceik_parms_struct, member), 0}
#define PS(sec, nm, member) {sec, nm, K_STR, 0, offsetof(struct mceik_parms_struct, member), \
                             sizeof(((struct mceik_parms_struct *)0)->member)}
#define O(sec, nm, k, member) {sec, nm, k, 1, offsetof(mceik_mcmc_opts, member), 0}

static const struct key KEYS[] = {
    PS("general", "projnm", projnm),
    PS("general", "scratch_dir", scratch_dir),
    P("grid", "x0", K_DBL, x0), P("grid", "y0", K_DBL, y0), P("grid", "z0", K_DBL, z0),
    P("grid", "dx", K_DBL, dx), P("grid", "dy", K_DBL, dy), P("grid", "dz", K_DBL, dz),
    O("grid", "nx", K_INT, nx), O("grid", "ny", K_INT, ny), O("grid", "nz", K_INT, nz),
    P("grid", "ndivx", K_INT, ndivx), P("grid", "ndivy", K_INT, ndivy), P("grid", "ndivz", K_INT, ndivz),
    P("grid", "nrefx", K_INT, nrefx), P("grid", "nrefy", K_INT, nrefy), P("grid", "nrefz", K_INT, nrefz),
    O("grid", "tt_interp", K_INT, tt_interp),
    P("eikonal", "tol", K_DBL, eikparms.tol), P("eikonal", "maxit", K_INT, eikparms.maxit),
    O("eikonal", "precision", K_INT, precision), O("eikonal", "max_waves", K_INT, max_waves),
    PS("mcmc", "resdir", mcparms.resdir),
    P("mcmc", "nburnin", K_INT, mcparms.nburnIn), P("mcmc", "niter", K_INT, mcparms.niter),
    P("mcmc", "keepk", K_INT, mcparms.keepK),
    O("mcmc", "nchains", K_INT, nchains), O("mcmc", "chain_offset", K_INT, chain_offset),
    O("mcmc", "vmin", K_INT, vmin), O("mcmc", "vmax", K_INT, vmax), O("mcmc", "dvmax", K_INT, dvmax),
    O("mcmc", "seed", K_U32, seed), O("mcmc", "max_samples", K_INT, max_samples),
    O("mcmc", "device", K_INT, device),
    O("mcmc", "nphase", K_INT, nphase), O("mcmc", "vsmin", K_INT, vsmin), O("mcmc", "vsmax", K_INT, vsmax),
    O("mcmc", "mask_s", K_INT, mask_s),
};
#define NKEYS ((int)(sizeof(KEYS) / sizeof(KEYS[0])))

int mceik_parms_defaults(struct mceik_parms_struct *parms, mceik_mcmc_opts *opts)
{
    if (parms) {
        memset(parms, 0, sizeof(*parms));
        /* homog.c:73-89: 31 x 28 x 25 km at 1 km from the origin */
        parms->dx = parms->dy = parms->dz = 1000.0;
        parms->ndivx = parms->ndivy = parms->ndivz = 1;
        parms->nrefx = parms->nrefy = parms->nrefz = 1;
        parms->eikparms.tol = 1.e-8;
        parms->eikparms.maxit = 50;
        parms->mcparms.keepK = 1;
        strcpy(parms->projnm, "mceik");
        strcpy(parms->scratch_dir, "./");
        strcpy(parms->mcparms.resdir, "./");
    }
    if (opts) {
        memset(opts, 0, sizeof(*opts));
        opts->nx = 32; opts->ny = 29; opts->nz = 26;   /* (x1 - x0)/dx + 1, homog.c:87-89 */
        opts->nchains = 1;
        opts->vmin = 1500; opts->vmax = 9000; opts->dvmax = 50;
        opts->seed = 2016;                             /* homog.c:113 srand(2016) */
        opts->precision = 32;
    }
    return 0;
}

static void lower(char *s) { for (; *s; s++) *s = (char)tolower((unsigned char)*s); }

static char *trim(char *s)
{
    while (isspace((unsigned char)*s)) s++;
    char *e = s + strlen(s);
    while (e > s && isspace((unsigned char)e[-1])) *--e = '\0';
    return s;
}

/* key "section:name" (case-insensitive).  0 ok, 1 unknown key, 2 bad value. */
int mceik_parms_set(struct mceik_parms_struct *parms, mceik_mcmc_opts *opts, const char *key, const char *value)
{
    static const char *fcnm = "mceik_parms_set";
    if (!key || !value) return 1;
    char k[256];
    if (strlen(key) >= sizeof(k)) return 1;
    strcpy(k, key);
    lower(k);
    char *colon = strchr(k, ':');
    if (!colon) {
        fprintf(stderr, "%s: key %s must be section:name\n", fcnm, key);
        return 1;
    }
    *colon = '\0';
    const char *sec = trim(k), *name = trim(colon + 1);
    char vbuf[1024];
    if (strlen(value) >= sizeof(vbuf)) return 2;
    strcpy(vbuf, value);
    char *v = trim(vbuf);
    size_t n = strlen(v);
    if (n >= 2 && v[0] == '"' && v[n - 1] == '"') { v[n - 1] = '\0'; v++; }
    for (int i = 0; i < NKEYS; i++) {
        if (strcmp(KEYS[i].section, sec) || strcmp(KEYS[i].name, name)) continue;
        char *base = KEYS[i].in_opts ? (char *)opts : (char *)parms;
        if (!base) return 0;                       /* caller did not ask for this record */
        char *dst = base + KEYS[i].off, *end = NULL;
        errno = 0;
        switch (KEYS[i].kind) {
        case K_INT: {
            long x = strtol(v, &end, 0);
            if (end == v || *trim(end) || errno || x < INT_MIN || x > INT_MAX) goto bad;
            *(int *)dst = (int)x;
            break;
        }
        case K_U32: {
            long long x = strtoll(v, &end, 0);
            if (end == v || *trim(end) || errno || x < 0 || x > 0xffffffffLL) goto bad;
            *(unsigned *)dst = (unsigned)x;
            break;
        }
        case K_DBL: {
            double x = strtod(v, &end);
            if (end == v || *trim(end) || errno || !isfinite(x)) goto bad;
            *(double *)dst = x;
            break;
        }
        case K_STR:
            if (strlen(v) >= KEYS[i].cap) goto bad;
            strcpy(dst, v);
            break;
        }
        return 0;
    bad:
        fprintf(stderr, "%s: invalid value '%s' for %s:%s\n", fcnm, value, sec, name);
        return 2;
    }
    fprintf(stderr, "%s: unknown key %s:%s\n", fcnm, sec, name);
    return 1;
}

/* 0 ok; -1 cannot open; > 0 the 1-based line number of the first bad line. */
int mceik_parms_read(const char *path, struct mceik_parms_struct *parms, mceik_mcmc_opts *opts)
{
    static const char *fcnm = "mceik_parms_read";
    FILE *f = path ? fopen(path, "r") : NULL;
    if (!f) {
        fprintf(stderr, "%s: cannot open %s\n", fcnm, path ? path : "(null)");
        return -1;
    }
    char line[2048], sec[128] = "";
    int lineno = 0, rc = 0;
    while (fgets(line, sizeof(line), f)) {
        lineno++;
        /* strip comments outside quotes */
        int q = 0;
        for (char *c = line; *c; c++) {
            if (*c == '"') q = !q;
            else if (!q && (*c == ';' || *c == '#')) { *c = '\0'; break; }
        }
        char *s = trim(line);
        if (!*s) continue;
        if (*s == '[') {
            char *e = strchr(s, ']');
            if (!e || *trim(e + 1) || (size_t)(e - s - 1) >= sizeof(sec)) { rc = lineno; break; }
            *e = '\0';
            strcpy(sec, trim(s + 1));
            continue;
        }
        char *eq = strchr(s, '=');
        if (!eq || !*sec) {
            fprintf(stderr, "%s: %s:%d: expected key = value inside a [section]\n", fcnm, path, lineno);
            rc = lineno;
            break;
        }
        *eq = '\0';
        char key[512];
        if (snprintf(key, sizeof(key), "%s:%s", sec, trim(s)) >= (int)sizeof(key)) { rc = lineno; break; }
        if (mceik_parms_set(parms, opts, key, eq + 1)) {
            fprintf(stderr, "%s: %s:%d: rejected\n", fcnm, path, lineno);
            rc = lineno;
            break;
        }
    }
    fclose(f);
    return rc;
}

/* Applies every argument of the form [--]section:key=value (and
 * --config=FILE / --config FILE, read first in argument order); other
 * arguments are left alone.  Returns the number of arguments consumed, or
 * -1 on the first bad one. */
int mceik_parms_args(int argc, char **argv, struct mceik_parms_struct *parms, mceik_mcmc_opts *opts)
{
    int used = 0;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (!a) continue;
        while (*a == '-') a++;
        if (!strncmp(a, "config", 6) && (a[6] == '=' || a[6] == '\0') && a != argv[i]) {
            const char *file = a[6] == '=' ? a + 7 : (i + 1 < argc ? argv[++i] : NULL);
            if (!file || mceik_parms_read(file, parms, opts)) return -1;
            used += a[6] == '=' ? 1 : 2;
            continue;
        }
        const char *eq = strchr(a, '='), *colon = strchr(a, ':');
        if (!eq || !colon || colon > eq) continue;
        char key[512];
        size_t n = (size_t)(eq - a);
        if (n >= sizeof(key)) return -1;
        memcpy(key, a, n);
        key[n] = '\0';
        if (mceik_parms_set(parms, opts, key, eq + 1)) return -1;
        used++;
    }
    return used;
}

/* Writes every key in INI form (a run's record next to its results). */
int mceik_parms_write(const char *path, const struct mceik_parms_struct *parms, const mceik_mcmc_opts *opts)
{
    FILE *f = path ? fopen(path, "w") : NULL;
    if (!f) return -1;
    const char *cur = "";
    for (int i = 0; i < NKEYS; i++) {
        const char *base = KEYS[i].in_opts ? (const char *)opts : (const char *)parms;
        if (!base) continue;
        if (strcmp(cur, KEYS[i].section)) {
            fprintf(f, "%s[%s]\n", *cur ? "\n" : "", KEYS[i].section);
            cur = KEYS[i].section;
        }
        const char *src = base + KEYS[i].off;
        switch (KEYS[i].kind) {
        case K_INT: fprintf(f, "%s = %d\n", KEYS[i].name, *(const int *)src); break;
        case K_U32: fprintf(f, "%s = %u\n", KEYS[i].name, *(const unsigned *)src); break;
        case K_DBL: fprintf(f, "%s = %.17g\n", KEYS[i].name, *(const double *)src); break;
        case K_STR: fprintf(f, "%s = \"%s\"\n", KEYS[i].name, src); break;
        }
    }
    return fclose(f) ? -1 : 0;
}
