/*
 * golden_io.h — tiny self-describing binary container for golden vectors (test infrastructure).
 * File = "SVTG" + u32 version, then records:
 *   u16 name_len, name, u8 dtype ('B','b','H','h','I','i','Q','q','d'), u8 ndim, u32 dims[ndim], data.
 * Read back by tests/golden_io.py.
 */
#ifndef GOLDEN_IO_H
#define GOLDEN_IO_H
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct GoldenFile {
    FILE *fp;
} GoldenFile;

static inline GoldenFile golden_open(const char *path) {
    GoldenFile g;
    g.fp = fopen(path, "wb");
    if (!g.fp) {
        fprintf(stderr, "cannot open %s\n", path);
        exit(2);
    }
    fwrite("SVTG", 1, 4, g.fp);
    uint32_t ver = 1;
    fwrite(&ver, 4, 1, g.fp);
    return g;
}

static inline size_t golden_dsize(char dt) {
    switch (dt) {
    case 'B':
    case 'b': return 1;
    case 'H':
    case 'h': return 2;
    case 'I':
    case 'i': return 4;
    default: return 8;
    }
}

static inline void golden_put(GoldenFile *g, const char *name, char dt, int ndim, const uint32_t *dims,
                              const void *data) {
    uint16_t nl = (uint16_t)strlen(name);
    fwrite(&nl, 2, 1, g->fp);
    fwrite(name, 1, nl, g->fp);
    uint8_t d = (uint8_t)dt, nd = (uint8_t)ndim;
    fwrite(&d, 1, 1, g->fp);
    fwrite(&nd, 1, 1, g->fp);
    size_t n = 1;
    for (int i = 0; i < ndim; i++) {
        fwrite(&dims[i], 4, 1, g->fp);
        n *= dims[i];
    }
    fwrite(data, golden_dsize(dt), n, g->fp);
}

static inline void golden_put1(GoldenFile *g, const char *name, char dt, uint32_t n0, const void *data) {
    golden_put(g, name, dt, 1, &n0, data);
}
static inline void golden_put2(GoldenFile *g, const char *name, char dt, uint32_t n0, uint32_t n1,
                               const void *data) {
    uint32_t d[2] = {n0, n1};
    golden_put(g, name, dt, 2, d, data);
}
static inline void golden_close(GoldenFile *g) { fclose(g->fp); }

/* SplitMix64: deterministic, platform-independent input stream */
typedef struct Rng {
    uint64_t s;
} Rng;
static inline uint64_t rng_next(Rng *r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint32_t rng_below(Rng *r, uint32_t n) { return (uint32_t)(rng_next(r) % n); }

#endif
