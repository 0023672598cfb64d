/* rt_par_write.h -- parallel, order-preserving text writer (par_write.c). */
#ifndef RT_PAR_WRITE_H
#define RT_PAR_WRITE_H

#include <stddef.h>
#include <stdio.h>

/* upper bound of the bytes one unit formats to (an object header block or
 * one line) */
#define RT_UNIT_MAX 1024

/* Formats unit j (0 = the header block, then its lines) of object o at p;
 * returns the bytes written (<= RT_UNIT_MAX, no terminating NUL counted). */
typedef size_t (*rt_unit_fmt)(const void *ctx, size_t o, size_t j, char *p);

/* Writes the units of objects 0..nobj-1 (units[o] each) to f in order,
 * formatted by the host threads (rt_host_threads()). */
int rt_par_write(FILE *f, const void *ctx, size_t nobj, const size_t *units, rt_unit_fmt fmt);

#endif
