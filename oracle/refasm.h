/* oracle/refasm.h -- TEST INFRASTRUCTURE ONLY (see refasm.c header). */
#ifndef EULERHIP_ORACLE_REFASM_H
#define EULERHIP_ORACLE_REFASM_H
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_WANT_DICT 1u  /* also return build()'s ordered dict */

typedef struct {
    uint64_t n_positions;     /* forward k-mer windows P over all N-split segments      */
    uint64_t n_dict;          /* entries of build()'s dict (strand-specific, ordered)   */
    char *dict_kmers;         /* n_dict * k chars, insertion order                       */
    uint32_t *dict_counts;    /* n_dict                                                  */
    uint64_t n_contigs;
    char *contig_chars;       /* contigs concatenated, all_contigs() order               */
    uint64_t *contig_offsets; /* n_contigs + 1                                           */
    uint64_t *link_offsets;   /* 2*n_contigs + 1: list 2i = G[i][0], 2i+1 = G[i][1]      */
    int64_t *links;           /* entry = 2*j + (orientation == '-')                      */
} oracle_result;

/* returns 0 on success, -1 bad argument, -3 out of memory, -4 a contig walk that the reference
 * would never finish (reads with bytes outside {A,C,G,T,N} only: see refasm_str.c) */
int oracle_assemble(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                    unsigned flags, oracle_result *out);
/* the same result from `threads` host threads: map -> reduceByKey counting as
 * src/ref_spark.py:76-84, all_contigs single-threaded (BASELINE.md §3 N-core baseline) */
int oracle_assemble_mt(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                       unsigned flags, int threads, oracle_result *out);
void oracle_free(oracle_result *r);
/* the string-keyed restatement (any bytes; refasm_str.c), also reached through the two above */
int oracle_assemble_str(const char *buf, const uint64_t *offsets, uint64_t nreads, int k, int limit,
                        unsigned flags, oracle_result *out);
const char *oracle_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
