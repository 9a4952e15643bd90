/* One build through the C ABI from plain C (no Python, no torch): the calls a reference-side
 * binding makes.  Reads a FASTA file, builds the BOSS chunk on device 0 with
 * IBOSSChunkConstructor::initialize's parameters (boss_chunk_construct.cpp:1134-1178), and compares
 * W, packed last, F and weights with a fixture written by tests/golden/make_capi_fixture.py.
 * Usage: capi_min <reads.fa> <k_b> <canonical 0|1> <bits_per_count> <fixture.bin>
 * Exit status 0 = identical, 1 = different, 2 = usage / I/O / library error. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mtg_boss.h"

static char *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = malloc((size_t)n + 1);
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) {
        fclose(f);
        free(buf);
        return NULL;
    }
    fclose(f);
    buf[n] = 0;
    *len = (size_t)n;
    return buf;
}

/* FASTA records -> one buffer of sequences back to back + offsets (header lines dropped,
 * sequence lines joined) */
static size_t parse_fasta(const char *text, size_t len, char **data, uint64_t **offsets) {
    char *out = malloc(len + 1);
    uint64_t *off = malloc((len / 2 + 2) * sizeof(uint64_t));
    size_t n = 0, o = 0, i = 0;
    while (i < len) {
        size_t e = i;
        while (e < len && text[e] != '\n') ++e;
        size_t le = e;
        if (le > i && text[le - 1] == '\r') --le;
        if (text[i] == '>') {
            off[n++] = o;
        } else if (n) {
            memcpy(out + o, text + i, le - i);
            o += le - i;
        }
        i = e + 1;
    }
    off[n] = o;
    *data = out;
    *offsets = off;
    return n;
}

int main(int argc, char **argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s reads.fa k_b canonical bits_per_count fixture.bin\n", argv[0]);
        return 2;
    }
    size_t flen = 0, xlen = 0;
    char *fa = slurp(argv[1], &flen);
    char *fx = slurp(argv[5], &xlen);
    if (!fa || !fx) {
        fprintf(stderr, "cannot read inputs\n");
        return 2;
    }
    char *data;
    uint64_t *offsets;
    const size_t n = parse_fasta(fa, flen, &data, &offsets);

    mtg_boss_params p;
    memset(&p, 0, sizeof p);
    p.k = strtoull(argv[2], NULL, 10);
    p.both_strands = atoi(argv[3]);
    p.bits_per_count = (uint8_t)atoi(argv[4]);
    p.num_threads = 4;
    p.container_type = MTG_CONTAINER_VECTOR;
    p.device_id = 0;
    mtg_boss_ctor *ctor = mtg_boss_ctor_create(&p);
    if (!ctor) {
        fprintf(stderr, "create: %s\n", mtg_last_error());
        return 2;
    }
    mtg_boss_chunk c;
    if (mtg_boss_ctor_add_packed(ctor, data, offsets, NULL, n) != MTG_OK ||
        mtg_boss_ctor_build_chunk(ctor, &c) != MTG_OK) {
        fprintf(stderr, "build: %s\n", mtg_last_error());
        return 2;
    }

    /* fixture: "MTGF", u64 n, u64 F[5], W[n], last words[(n + 63) / 64], weights u32[n] if bits */
    int same = xlen >= 52 && memcmp(fx, "MTGF", 4) == 0;
    uint64_t fn = 0, fF[5];
    if (same) {
        memcpy(&fn, fx + 4, 8);
        memcpy(fF, fx + 12, 40);
        same = fn == c.n && memcmp(fF, c.F, 40) == 0;
    }
    const uint64_t nw = (c.n + 63) / 64;
    const size_t need = 52 + c.n + nw * 8 + (c.weights ? c.n * 4 : 0);
    same = same && xlen == need;
    if (same) same = memcmp(fx + 52, c.W, c.n) == 0;
    if (same) same = memcmp(fx + 52 + c.n, c.last, nw * 8) == 0;
    if (same && c.weights) same = memcmp(fx + 52 + c.n + nw * 8, c.weights, c.n * 4) == 0;
    printf("capi_min: %lu sequences, %lu rows, k=%lu, %s\n", (unsigned long)n, (unsigned long)c.n,
           (unsigned long)c.k, same ? "identical to the fixture" : "DIFFERENT from the fixture");
    mtg_boss_chunk_free(&c);
    mtg_boss_ctor_destroy(ctor);
    free(data);
    free(offsets);
    free(fa);
    free(fx);
    return same ? 0 : 1;
}
