/* os.c -- include/os.h: the reference's file-system helpers (its os.h,
 * declared by its mceik.h), so a harness that includes mceik.h for them links
 * unchanged.  Plain POSIX. */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "../../include/os.h"

bool os_path_exists(const char *pathnm)
{
    struct stat s;
    return pathnm && pathnm[0] && stat(pathnm, &s) == 0;
}

bool os_path_isdir(const char *dirnm)
{
    struct stat s;
    return dirnm && dirnm[0] && stat(dirnm, &s) == 0 && S_ISDIR(s.st_mode);
}

bool os_path_isfile(const char *filenm)
{
    struct stat s;
    return filenm && filenm[0] && stat(filenm, &s) == 0 && S_ISREG(s.st_mode);
}

int os_mkdir(const char *dirnm)
{
    if (!dirnm || !dirnm[0]) return -1;
    if (mkdir(dirnm, 0777) != 0) {
        printf("os_mkdir: Error making directory: %s\n", dirnm);
        return -1;
    }
    return 0;
}

int os_makedirs(const char *path)
{
    if (!path || !path[0]) return -1;
    if (os_path_isdir(path)) return 0;
    char *work = strdup(path);
    if (!work) return -1;
    int rc = 0;
    /* every prefix ending before a '/' (and the whole path), parents first */
    for (char *p = work + 1;; p++) {
        const char c = *p;
        if (c != '/' && c != '\0') continue;
        *p = '\0';
        if (!os_path_isdir(work) && mkdir(work, 0777) != 0 && errno != EEXIST) {
            printf("os_makedirs: Error making directory: %s\n", work);
            rc = -1;
        }
        *p = c;
        if (rc || c == '\0') break;
    }
    free(work);
    return rc == 0 && os_path_isdir(path) ? 0 : -1;
}
