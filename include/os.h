/*
 * os.h -- the file-system helpers the reference's include/os.h declares
 * (its mceik.h includes this header; implemented in libmceik_hip.so,
 * csrc/os.c).  Guard as the reference's (_os_os_h__).
 */
#ifndef _os_os_h__
#define _os_os_h__ 1
#include <stdbool.h>
#ifdef __cplusplus
extern "C" {
#endif
/* true if pathnm names an existing file-system entry */
bool os_path_exists(const char *pathnm);
/* true if dirnm is an existing directory */
bool os_path_isdir(const char *dirnm);
/* true if filenm is an existing regular file */
bool os_path_isfile(const char *filenm);
/* makes path and its missing parents (0 ok or already a directory, -1 error) */
int os_makedirs(const char *path);
/* makes one directory (0 ok, -1 error, e.g. it exists or the parent does not) */
int os_mkdir(const char *dirnm);
#ifdef __cplusplus
}
#endif
#endif /* _os_os_h__ */
