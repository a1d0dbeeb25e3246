/*
 * oracle/zrealloc.c -- TEST INFRASTRUCTURE ONLY: an LD_PRELOAD shim used when
 * capturing transform goldens from the reference binary.  The reference prints
 * each chromosome's tf_buffer with "%s" although realloc() never NUL-terminates
 * it (hpp:413-425, hpp:395); with a zero-filling realloc the dump stops exactly
 * at tf_buffer_size.  The reference is not modified.
 */
#define _GNU_SOURCE
#include <malloc.h>
#include <stdlib.h>
#include <string.h>

void* realloc(void* old, size_t n)
{
    void* p = malloc(n + 64);
    if (!p) return NULL;
    memset(p, 0, n + 64);
    if (old) {
        size_t have = malloc_usable_size(old);
        memcpy(p, old, have < n ? have : n);
        free(old);
    }
    return p;
}
