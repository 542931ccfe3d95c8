/*
 * oracle/refasm.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, single-threaded restatement of the reference CPU de Bruijn assembler
 *   /root/reference/src/referenceassembler/referenceAssembler.py
 *     twin:7-10, kmers:12-14, fw/bw:16-22, build:25-42, contig_to_string:44-45,
 *     get_contig:47-56, get_contig_forward:59-77, all_contigs:79-111
 * (identical algorithm in /root/reference/tests/referenceAssembler.py:6-115, BASELINE config 1).
 *
 * It is the parity checker for the HIP path and the `cpu_baseline` leg of bench.py
 * (kind "port", 1 core).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load it; the product library (libeulerhip.so) never does.
 *
 * Pinned: tests/test_oracle.py checks it against every golden vector generated from the
 * real reference (the JSON fixtures in tests/golden/, made by tests/golden/make_golden.py).
 *
 * Alphabet: over {A,C,G,T,N} k-mers are 2-bit packed (A=0,C=1,G=2,T=3, first base most
 * significant); 'N' splits a read into segments exactly like `read.split('N')` (build:29).
 * k <= 32 uses 64-bit keys, 32 < k <= 64 uses 128-bit keys.  Reads holding any other byte
 * (lowercase, IUPAC codes: the reference keeps them as opaque symbols, twin:7-10) go to the
 * string-keyed restatement in refasm_str.c.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

#include "refasm.h"

typedef unsigned __int128 u128;

static __thread char g_err[256];
const char *oracle_last_error(void) { return g_err; }
void oracle_set_error(const char *msg) { snprintf(g_err, sizeof g_err, "%s", msg); }

int oracle_assemble_str(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                        unsigned flags, oracle_result *out);


static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}

static inline int base_code(unsigned char c) {
    switch (c) {
    case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
    case 'N': return -1;
    default: return -2;
    }
}

/* a byte outside {A,C,G,T,N} in the reads: the string-keyed restatement */
static int extended_alphabet(const char *buf, const uint64_t *offsets, uint64_t nreads) {
    if (!nreads) return 0;
    for (uint64_t i = offsets[0]; i < offsets[nreads]; i++)
        if (base_code((unsigned char)buf[i]) == -2) return 1;
    return 0;
}

/* two instantiations: KEY = uint64_t (k <= 32) and KEY = u128 (k <= 64) */
#define KEY uint64_t
#define SFX _64
#define KHASH(x) mix64(x)
#include "refasm_impl.h"
#undef KEY
#undef SFX
#undef KHASH

#define KEY u128
#define SFX _128
#define KHASH(x) mix64((uint64_t)(x) ^ mix64((uint64_t)((x) >> 64)))
#include "refasm_impl.h"
#undef KEY
#undef SFX
#undef KHASH

int oracle_assemble(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                    unsigned flags, oracle_result *out) {
    memset(out, 0, sizeof(*out));
    if (k < 1 || k > 64) { snprintf(g_err, sizeof g_err, "k=%d out of range [1,64]", k); return -1; }
    if (extended_alphabet(buf, offsets, nreads)) return oracle_assemble_str(buf, offsets, nreads, k, limit, flags, out);
    if (k <= 32) return assemble_64(buf, offsets, nreads, k, limit, flags, out);
    return assemble_128(buf, offsets, nreads, k, limit, flags, out);
}

int oracle_assemble_mt(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                       unsigned flags, int threads, oracle_result *out) {
    memset(out, 0, sizeof(*out));
    if (k < 1 || k > 64) { snprintf(g_err, sizeof g_err, "k=%d out of range [1,64]", k); return -1; }
    if (extended_alphabet(buf, offsets, nreads)) return oracle_assemble_str(buf, offsets, nreads, k, limit, flags, out);
    if (k <= 32) return assemble_mt_64(buf, offsets, nreads, k, limit, flags, threads, out);
    return assemble_mt_128(buf, offsets, nreads, k, limit, flags, threads, out);
}

void oracle_free(oracle_result *r) {
    free(r->dict_kmers); free(r->dict_counts);
    free(r->contig_chars); free(r->contig_offsets);
    free(r->link_offsets); free(r->links);
    memset(r, 0, sizeof(*r));
}
