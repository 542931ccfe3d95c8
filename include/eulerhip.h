/*
 * eulerhip.h -- C ABI of libeulerhip.so, the MI355X (gfx950) de Bruijn + Euler-tour core.
 *
 * Plain `extern "C"`, plain pointers and sizes, int status (EC_OK = 0), thread-local
 * ec_last_error().  Two layers:
 *
 *  1. The fused, device-resident production path (ec_session + ec_assemble_*), a drop-in
 *     for the reference's CPU assembler build()+all_contigs()
 *     (src/referenceassembler/referenceAssembler.py:25-111 and the identical
 *     tests/referenceAssembler.py:23-115 named by BASELINE config 1), which is also what the
 *     reference GPU orchestration assemble2() (src/eulercuda.py:448-504) is meant to compute.
 *     Contigs, their order and the GFA link table are bit-identical to the reference.
 *
 *  2. Per-module drop-ins for the reference's PyCUDA module functions (host buffers in and
 *     out, like the reference's drv.In / .get() round trips).  Each declaration cites the
 *     reference function it replaces.
 *
 * k-mer codes are 2-bit, MSB-first (A=0 C=1 G=2 T=3), exactly the reference encoding
 * (src/pyencode.py:40,62-69).  Reads are ASCII over {A,C,G,T,N}; 'N' splits a read into
 * segments (referenceAssembler.py:29).  Other bytes -> EC_ERR_ALPHABET.
 */
#ifndef EULERHIP_H
#define EULERHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define EC_OK 0
#define EC_ERR_ARG (-1)      /* bad argument (k range, null pointer, size)                   */
#define EC_ERR_ALPHABET (-2) /* read byte outside {A,C,G,T,N}                                 */
#define EC_ERR_NOMEM (-3)    /* device or host allocation failed                              */
#define EC_ERR_HIP (-4)      /* HIP runtime error (message in ec_last_error)                  */
#define EC_ERR_CAPACITY (-5) /* table overflow that survived the retries                       */
#define EC_ERR_STATE (-6)    /* result requested before a successful ec_assemble_*            */

#define EC_MAX_K 32 /* fused path: k <= 32 (64-bit keys) */

const char *ec_last_error(void);
int ec_version(void); /* major*10000 + minor*100 + patch */

/* ---- layer 1: fused device-resident assembly ------------------------------------------- */
typedef struct ec_session ec_session;

#define EC_FLAG_WANT_DICT 1u /* also keep build()'s ordered dict for ec_copy_dict */
#define EC_FLAG_TIMING 2u    /* record per-stage HIP-event times (ec_stats.stage_ms) */
#define EC_FLAG_GENERAL 4u   /* force the general (single HBM hash table) counting path */

#define EC_NSTAGES 8
/* stage ids for ec_stats.stage_ms / ec_stage_name */
#define EC_STAGE_PRESCAN 0 /* alphabet check, positions, HyperLogLog distinct estimate  */
#define EC_STAGE_COUNT 1   /* encode + canonical count + first-occurrence (build:25-35)  */
#define EC_STAGE_COMPACT 2 /* solid filter count > limit + compaction (build:37-39)      */
#define EC_STAGE_LINKS 3   /* 8 neighbour probes, unitig successor links (get_contig_forward:59-77) */
#define EC_STAGE_RANK 4    /* pointer-jumping list ranking of paths / cycles             */
#define EC_STAGE_STARTS 5  /* component start = first dict entry, contig order (all_contigs:82-88) */
#define EC_STAGE_EMIT 6    /* contig strings (contig_to_string:44-45)                     */
#define EC_STAGE_GFA 7     /* GFA link table G (all_contigs:90-109)                       */

#define EC_NKERNELS 5
/* kernel ids for ec_stats.kernel_ms (EC_FLAG_TIMING) */
#define EC_KERNEL_UPSWEEP 0   /* encode pass 1: alphabet, P, HyperLogLog, bucket histogram   */
#define EC_KERNEL_DOWNSWEEP 1 /* encode pass 2: 16-B k-mer records scattered by bucket       */
#define EC_KERNEL_BUCKET 2    /* per-bucket LDS counting + solid filter + compaction          */
#define EC_KERNEL_COUNT 3     /* general path: HBM hash-table counting                        */
#define EC_KERNEL_REFINE 4    /* split coarse bucket runs into final buckets (LDS sort)       */

#define EC_PATH_PARTITIONED 0 /* radix-partitioned LDS counting (count_part.h)               */
#define EC_PATH_GENERAL 1     /* single HBM hash table (count_global.h)                      */

typedef struct {
    uint64_t n_reads;
    uint64_t n_positions;    /* P: forward k-mer windows over all N-split segments            */
    uint64_t n_distinct_est; /* HyperLogLog estimate of distinct canonical k-mers             */
    uint64_t n_distinct;     /* distinct canonical k-mers counted                              */
    uint64_t n_solid;        /* U: canonical k-mers with dict count > limit                    */
    uint64_t n_dict;         /* len(build()) = strand-specific entries (2U minus palindromes)  */
    uint64_t n_contigs;
    uint64_t n_contig_chars;
    uint64_t n_links;
    uint64_t table_capacity; /* general path: HBM hash slots; partitioned: buckets * LDS slots */
    uint64_t n_rulers;       /* sparse ruling-set size used by the list ranking               */
    uint32_t table_retries;
    uint32_t rank_rounds;    /* Wyllie rounds on the ruler list                               */
    uint32_t count_path;     /* EC_PATH_*                                                     */
    uint32_t n_buckets;      /* partitioned path: B                                           */
    float stage_ms[EC_NSTAGES];   /* EC_FLAG_TIMING only */
    float kernel_ms[EC_NKERNELS]; /* EC_FLAG_TIMING only */
} ec_stats;

int ec_session_create(ec_session **out, int device);
/* run on this hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = own stream */
int ec_session_set_stream(ec_session *s, void *hip_stream);
int ec_session_destroy(ec_session *s);

/* Reads already resident in device memory: d_reads = concatenated ASCII, d_offsets[nreads+1]
 * = byte offsets (uint64).  limit: keep k-mers whose dict count > limit (build(limit=1)). */
int ec_assemble_device(ec_session *s, const uint8_t *d_reads, const uint64_t *d_offsets,
                       uint64_t nreads, int k, int limit, unsigned flags);
/* Same on host buffers (copies H2D first). */
int ec_assemble_host(ec_session *s, const uint8_t *reads, uint64_t nbytes, const uint64_t *offsets,
                     uint64_t nreads, int k, int limit, unsigned flags);

int ec_get_stats(ec_session *s, ec_stats *out);
const char *ec_stage_name(int stage);
/* contigs: chars[n_contig_chars], offsets[n_contigs+1] (all_contigs r, in order) */
int ec_copy_contigs(ec_session *s, char *chars, uint64_t *offsets);
/* GFA links: link_offsets[2*n_contigs+1]; list 2i = G[i][0], 2i+1 = G[i][1];
 * links[n_links] entry = 2*j + (orientation == '-') */
int ec_copy_links(ec_session *s, uint64_t *link_offsets, int64_t *links);
/* ordered dict of build(): kmers[n_dict*k] chars, counts[n_dict]; needs EC_FLAG_WANT_DICT */
int ec_copy_dict(ec_session *s, char *kmers, uint32_t *counts);

/* ---- read-sharded multi-GPU building blocks (pycuda-euler_amd/distributed.py) ------------
 * Replace the reference's distribution layer (Spark mapPartitions of assemble2,
 * src/cli_spark_gpu.py:37, and the reduceByKey k-mer shuffle of src/ref_spark.py:83-84) with
 * count-local -> all-to-all by owner -> merge + solid filter -> all-gather -> graph phase.
 * All record buffers are device memory of ec_kmer_record (32 B). */
typedef struct {
    uint64_t key;   /* canonical 2-bit k-mer                                                */
    uint32_t count; /* dict count contribution (palindromes count 2 per occurrence)          */
    uint32_t pad;
    uint64_t first_canon; /* first insertion event of the canonical string: read << 32 | local */
    uint64_t first_twin;  /* first insertion event of its twin                                */
} ec_kmer_record;

/* count the shard (global read ids start at read_base); keeps every distinct k-mer */
int ec_count_shard(ec_session *s, const uint8_t *d_reads, const uint64_t *d_offsets, uint64_t nreads,
                   uint64_t read_base, int k, unsigned flags);
/* number of dense k-mer records the session holds (after ec_count_shard / ec_merge_owned) */
uint64_t ec_dense_count(ec_session *s);
/* pack the held records owner-major into d_out (ec_kmer_record[ec_dense_count]); owner_counts
 * (host, nowners <= 256) receives the records per owner.  d_out = NULL: counts only. */
int ec_export_by_owner(ec_session *s, int nowners, void *d_out, uint64_t *owner_counts);
/* owner side: aggregate received records, keep count > limit */
int ec_merge_owned(ec_session *s, const void *d_records, uint64_t n, int k, int limit, unsigned flags);
/* copy the held records (ec_merge_owned's solid set) to d_out */
int ec_export_dense(ec_session *s, void *d_out);
/* graph phase (links .. GFA) on a complete solid set; results via ec_copy_* */
int ec_assemble_from_solid(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags);

#ifdef __cplusplus
}
#endif
#endif /* EULERHIP_H */
