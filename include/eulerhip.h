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
 * (src/pyencode.py:40,62-69).  Reads are ASCII; 'N' splits a read into segments
 * (referenceAssembler.py:29).  Any other byte (lowercase, IUPAC codes) is an opaque symbol that
 * is its own complement, as the reference's twin() keeps it (:7-10): such inputs take the
 * extended-alphabet path (csrc/extended.h) with sb-bit symbol codes (sb = 4 / 5 / 8 for up to
 * 16 / 32 / 256 distinct symbols) and need sb * k <= 126, else EC_ERR_ALPHABET.
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
#define EC_ERR_ALPHABET (-2) /* extended alphabet: sb * k > 126 (see above)                    */
#define EC_ERR_NOMEM (-3)    /* device or host allocation failed                              */
#define EC_ERR_HIP (-4)      /* HIP runtime error (message in ec_last_error)                  */
#define EC_ERR_CAPACITY (-5) /* table overflow that survived the retries                       */
#define EC_ERR_STATE (-6)    /* result requested before a successful ec_assemble_*, or an
                              * extended-alphabet input on which the reference's
                              * get_contig_forward never returns (referenceAssembler.py:59-77) */

#define EC_MAX_K 63 /* k <= 32: 64-bit keys; 32 < k <= 63: 128-bit keys */

const char *ec_last_error(void);
int ec_version(void); /* major*10000 + minor*100 + patch */

/* ---- layer 1: fused device-resident assembly ------------------------------------------- */
typedef struct ec_session ec_session;

#define EC_FLAG_WANT_DICT 1u /* also keep build()'s ordered dict for ec_copy_dict */
#define EC_FLAG_TIMING 2u    /* record per-stage and per-kernel HIP-event times (stage_ms, kernel_ms) */
#define EC_FLAG_KERNEL_TIMING 128u /* per-kernel HIP-event times only (kernel_ms): 6-10 events a call
                                     * instead of ~26, for timed benchmark steps */
#define EC_FLAG_GENERAL 4u   /* force the general (single HBM hash table) counting path */
#define EC_FLAG_WIDE_RECORDS 8u /* partitioned path: 16-B window records only (default for k < 21 or
                                  * reads with N: 12-B records when every read is N-free and of one length) */
#define EC_FLAG_WINDOW_RECORDS 16u /* partitioned path: one record per k-mer window, never super-k-mers
                                    * (never count_sk2.h's default 16-B super-k-mer records) */
#define EC_FLAG_EXACT_COUNT 64u /* partitioned path: histogram-sized runs only (count_part.h), never the
                                  * fixed-capacity runs of count_v2.h */
#define EC_FLAG_SUPERKMER 32u /* accepted and ignored: super-k-mer records (count_sk2.h, ec_stats.count_variant 3)
                                * are the default where they apply -- N-free reads of one length,
                                * 21 <= k <= 32; the 32-B record path this flag selected was removed */

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
#define EC_PATH_SUPERKMER 2   /* no longer reported (the 32-B super-k-mer path was removed)     */

typedef struct {
    uint64_t n_reads;
    uint64_t n_positions;    /* P: forward k-mer windows over all N-split segments            */
    uint64_t n_distinct_est; /* HyperLogLog estimate of distinct canonical k-mers             */
    uint64_t n_distinct;     /* distinct canonical k-mers counted (an estimate, +-2 %, when the
                              * seen-twice filter buckets of error-rich inputs drop singletons) */
    uint64_t n_solid;        /* U: canonical k-mers with dict count > limit                    */
    uint64_t n_dict;         /* len(build()) = strand-specific entries (2U minus palindromes)  */
    uint64_t n_contigs;
    uint64_t n_contig_chars;
    uint64_t n_links;
    uint64_t table_capacity; /* general path: HBM hash slots; partitioned: buckets * LDS slots */
    uint64_t n_rulers;       /* sparse ruling-set size used by the list ranking               */
    uint64_t n_records;      /* partitioned paths: records moved (P windows, or super-k-mers)  */
    uint32_t table_retries;
    uint32_t rank_rounds;    /* Wyllie rounds on the ruler list                               */
    uint32_t count_path;     /* EC_PATH_*                                                     */
    uint32_t n_buckets;      /* partitioned path: B                                           */
    uint32_t record_bytes;   /* partitioned paths: 10 / 12 / 16 per window record, 16 or 32 per
                              * super-k-mer                                                   */
    uint32_t count_variant;  /* partitioned path: 0 = histogram-sized runs (count_part.h),
                              * 1 = fixed-capacity runs without the upsweep (count_v2.h), 12-B
                              * records; 2 = the same with 10-B records (hashed-key remnants);
                              * 3 = 16-B super-k-mer records on fixed-capacity runs
                              * (count_sk2.h; the default for N-free reads of one length,
                              * 21 <= k <= 32, inputs that need no seen-twice filter)          */
    float stage_ms[EC_NSTAGES];   /* EC_FLAG_TIMING only */
    float kernel_ms[EC_NKERNELS]; /* EC_FLAG_TIMING or EC_FLAG_KERNEL_TIMING */
} ec_stats;

int ec_session_create(ec_session **out, int device);
/* run on this hipStream_t, e.g. torch.cuda.current_stream().cuda_stream (NULL = the null stream,
 * torch's default); EC_OWN_STREAM = back to a non-blocking stream owned by the session (the
 * state after ec_session_create).  Inputs produced asynchronously on another stream must be
 * complete (or that stream must be this one) when an ec_* call starts. */
#define EC_OWN_STREAM ((void *)-1)
int ec_session_set_stream(ec_session *s, void *hip_stream);
int ec_session_destroy(ec_session *s);
/* Device memory held by the session buffers of this process (bytes) and its high-water mark;
 * reset != 0 restarts the mark at the current holding after reading it.  EULERHIP_MEMLOG=1
 * logs every buffer of >= 1 GB to stderr as it is allocated. */
int ec_mem_stats(uint64_t *held, uint64_t *peak, int reset);
/* Release the session's device buffers of at least min_bytes (0: all but its scalars) and every
 * device state they held (dense k-mer arrays, a loaded or placed graph): the next call starts
 * from its inputs; results already copied to host memory stay fetchable.  The sharded path
 * calls it after a large shard's export, so the owner merge and graph phase get the count's
 * memory (distributed.py). */
int ec_session_trim(ec_session *s, uint64_t min_bytes);
/* Device bytes the session's buffers hold. */
uint64_t ec_session_bytes(ec_session *s);

/* Reads already resident in device memory: d_reads = concatenated ASCII, d_offsets[nreads+1]
 * = byte offsets (uint64).  limit: keep k-mers whose dict count > limit (build(limit=1)). */
int ec_assemble_device(ec_session *s, const uint8_t *d_reads, const uint64_t *d_offsets,
                       uint64_t nreads, int k, int limit, unsigned flags);
/* Same on host buffers: the reference's entry (src/eulercuda.py:484-497 hands the host read
 * buffer to encode_lmer_device, src/pyencode.py:14, which copies it H2D).  The reads are copied
 * in chunks on a second stream while the super-k-mer partition runs on the chunks that have
 * arrived; pinned (page-locked) host memory copies at the full PCIe rate. */
int ec_assemble_host(ec_session *s, const uint8_t *reads, uint64_t nbytes, const uint64_t *offsets,
                     uint64_t nreads, int k, int limit, unsigned flags);

/* 2-bit packed host reads (a quarter of ec_assemble_host's PCIe bytes).  Layout: base i of the
 * concatenated reads at bits 2 (i & 3) of codes[i >> 2] (A=0 C=1 G=2 T=3); every byte that is not
 * A, C, G or T ('N', anything else) is an exception: exc_pos[] ascending base positions, exc_byte[]
 * the original bytes (their code bits are ignored).  Read r = bases [offsets[r], offsets[r+1]),
 * or, offsets = NULL, [r * read_len, (r + 1) * read_len).  Results equal ec_assemble_host's on
 * the unpacked reads. */
int ec_assemble_packed_host(ec_session *s, const uint8_t *codes, uint64_t nbases, const uint64_t *offsets,
                            uint64_t nreads, uint32_t read_len, const uint64_t *exc_pos, const uint8_t *exc_byte,
                            uint64_t n_exc, int k, int limit, unsigned flags);
/* Staged packed batches (round 4): a pipeline over consecutive read batches.  ec_stage_packed_host
 * queues one batch's H2D copies (same arguments as ec_assemble_packed_host; the host buffers must
 * stay valid and unchanged until the batch is assembled) into one of two device slots and returns
 * at once; ec_assemble_staged assembles the oldest staged batch (results as ec_assemble_*).
 * Staging batch i + 1 before assembling batch i overlaps its PCIe copy with batch i's kernels:
 *   stage(b0); stage(b1); assemble -> b0; stage(b2); assemble -> b1; ...
 * EC_ERR_STATE: a third batch staged, or ec_assemble_staged with none (ec_assemble_packed_host
 * also refuses while batches are staged). */
int ec_stage_packed_host(ec_session *s, const uint8_t *codes, uint64_t nbases, const uint64_t *offsets,
                         uint64_t nreads, uint32_t read_len, const uint64_t *exc_pos, const uint8_t *exc_byte,
                         uint64_t n_exc);
int ec_assemble_staged(ec_session *s, int k, int limit, unsigned flags);
/* ASCII reads (CSR) -> that layout, on `threads` host threads (<= 0: up to 16).  codes holds
 * ceil(nbases / 4) bytes; exceptions beyond exc_cap are counted but not written (*n_exc = the
 * total: call again with a larger buffer when it exceeds exc_cap); *read_len = the common read
 * length, or 0 when the reads differ in length (offsets are then needed). */
int ec_pack_reads(const uint8_t *reads, const uint64_t *offsets, uint64_t nreads, int threads, uint8_t *codes,
                  uint64_t *exc_pos, uint8_t *exc_byte, uint64_t exc_cap, uint64_t *n_exc, uint32_t *read_len);

int ec_get_stats(ec_session *s, ec_stats *out);
const char *ec_stage_name(int stage);
/* contigs: chars[n_contig_chars], offsets[n_contigs+1] (all_contigs r, in order) */
int ec_copy_contigs(ec_session *s, char *chars, uint64_t *offsets);
/* GFA links: link_offsets[2*n_contigs+1]; list 2i = G[i][0], 2i+1 = G[i][1];
 * links[n_links] entry = 2*j + (orientation == '-') */
int ec_copy_links(ec_session *s, uint64_t *link_offsets, int64_t *links);
/* ordered dict of build(): kmers[n_dict*k] chars, counts[n_dict]; needs EC_FLAG_WANT_DICT */
int ec_copy_dict(ec_session *s, char *kmers, uint32_t *counts);

/* ---- layer 2: per-module drop-ins (host buffers, one H2D/D2H round trip per call) ---------
 * Each restates the INTENDED semantics of the reference PyCUDA function named; the reference's
 * out-of-bounds and race defects are fixed, flags reproduce them where a caller may
 * depend on them.  Struct layouts match the reference numpy dtypes (packed):
 *   EulerVertex {u64 vid; u32 ep, ecount, lp, lcount}   24 B  (src/pydebruijn.py:606)
 *   EulerEdge   {u64 eid; u32 v1, v2, s, pad}           24 B  (src/pydebruijn.py:604)
 *   Vertex      {u32 vid, n1, n2}                        12 B  (src/pyeulertour.py:734)
 *   CircuitEdge {u32 ceid, e1, e2, c1, c2}               20 B  (src/pyeulertour.py:785) */
#define EC_MOD_TAIL_DROP 1u  /* pygpuhash: floor(n/1024)-block grid drops the tail (src/pygpuhash.py:57-61) */
#define EC_MOD_REF_BOUNDS 2u /* pydebruijn: setupEdges' `< lmerCount` bounds (src/pydebruijn.py:449)     */
#define EC_MOD_SWIPE 4u      /* pyeulertour: run the commented-out swipe body (src/pyeulertour.py:539-552) */
#define EC_MOD_TREE_MARKS 8u /* pyeulertour: mark only the spanning tree's edges (mark starts at zero, not at
                              * one as :659; mark[e1] of each tree edge): with EC_MOD_SWIPE every connected
                              * component's circuits merge into one Euler tour */
#define EC_HASH_BUCKET_ITEMS 520 /* MAX_BUCKET_ITEM (src/pygpuhash.py:14) */

/* E1 encode_lmer_device (src/pyencode.py:14-98): out[p] = MSB-first 2-bit code of buf[p..p+L-1]
 * with the reference table codeF[c & 7] (N and '\n' -> A); bytes past the end read as 0 */
int ec_encode_lmers(const uint8_t *buf, uint64_t n, uint32_t L, uint64_t *out);
/* E2 compute_kmer_device (src/pyencode.py:101-159): pk = (x & (mask<<2)) >> 2, sk = x & mask */
int ec_split_kmers(const uint64_t *lmers, uint64_t n, uint64_t mask, uint64_t *pk, uint64_t *sk);
/* E3 compute_lmer_complement_device, intended (src/pyencode.py:162-232): sum codeR(c[p+i]) << 2i */
int ec_encode_lmers_rc(const uint8_t *buf, uint64_t n, uint32_t L, uint64_t *out);
/* H1-H5 create_hash_table_device (src/pygpuhash.py:261-314): nb = 0 -> n/409+1 buckets;
 * TK[nb*520], TV[nb*520] (bucket b, rank within the bucket), bucket_size[nb] */
uint32_t ec_hash_bucket_count(uint64_t n);
int ec_hash_build(const uint64_t *keys, const uint32_t *vals, uint64_t n, uint32_t nb, unsigned flags, uint64_t *TK,
                  uint32_t *TV, uint32_t *bucket_size);
/* H6 getHashValue (src/pydebruijn.py:56-87): out[i] = TV of keys[i] or 0xFFFFFFFF */
int ec_hash_lookup(const uint64_t *TK, const uint32_t *TV, const uint32_t *bucket_size, uint32_t nb,
                   const uint64_t *keys, uint64_t n, uint32_t *out);
/* G1-G5 construct_debruijn_graph_device (src/pydebruijn.py:515-619): ev[nk] EulerVertex,
 * ee/l/e[E] with E = sum(lmer_values) (*edge_count; ee_out = NULL -> sizing only) */
int ec_debruijn_build(const uint64_t *lmer_keys, const uint32_t *lmer_values, uint64_t nl, const uint64_t *kmer_keys,
                      uint64_t nk, uint32_t l, const uint64_t *TK, const uint32_t *TV, const uint32_t *bucket_size,
                      uint32_t nb, unsigned flags, void *ev_out, void *ee_out, uint32_t *l_out, uint32_t *e_out,
                      uint64_t *edge_count);
/* C1 find_component_device (src/pycomponent.py:668-723): D[i] = smallest vertex of i's
 * component over edges i-n1, i-n2 (fixpoint; the reference stops after one iteration) */
int ec_components(const void *vertices, uint64_t n, uint32_t *D);
/* T1-T3 findEulerDevice (src/pyeulertour.py:714-792): successors written into ee (in place),
 * circuit-graph edges (CircuitEdge[E] capacity, unsorted) and their / the circuit counts */
int ec_find_euler(const void *ev, uint64_t vcount, const uint32_t *l, const uint32_t *e, void *ee, uint64_t E,
                  void *cg_edges, uint64_t *cg_edge_count, uint32_t *cg_vertex_count);
/* T5 executeSwipeDevice (src/pyeulertour.py:656-664): mark (all ones, :659) + tree marks;
 * the swipe itself only with EC_MOD_SWIPE (a no-op in the reference; needs e to be a permutation) */
int ec_execute_swipe(const void *ev, uint64_t vcount, const uint32_t *e, void *ee, uint64_t E, const void *cg_edges,
                     uint64_t cg_edge_count, const uint32_t *tree, uint64_t tree_count, unsigned flags,
                     uint32_t *mark_out);
/* T4 findSpanningTree (src/eulercuda.py:266-305): the spanning forest of the circuit graph
 * (CircuitEdge[cg_edge_count], circuits 0..cg_vertex_count-1) that Kruskal takes in edge-index
 * order, as ascending circuit-edge indices in tree[*tree_count] (capacity cg_edge_count) */
int ec_spanning_forest(const void *cg_edges, uint64_t cg_edge_count, uint64_t cg_vertex_count, uint32_t *tree,
                       uint64_t *tree_count);
/* T6 identify_contig_start (src/pyeulertour.py:667-706): contig_start[ee[i].s] = 0 for s < E */
int ec_identify_contig_start(const void *ee, uint64_t E, uint32_t *contig_start);

/* step-level drop-ins for the reference's intermediate module functions */
/* phase1_device (src/pygpuhash.py:18-73): offset[i] = position of key i among the keys of its
 * bucket in input order (the reference's atomicInc order is arbitrary), bucket_size[nb] */
int ec_hash_phase1(const uint64_t *keys, uint64_t n, uint32_t nb, unsigned flags, uint32_t *offset,
                   uint32_t *bucket_size);
/* copy_to_bucket_device (src/pygpuhash.py:76-170): buf[start[bucket] + offset[i]] = key/value */
int ec_hash_copy_to_bucket(const uint64_t *keys, const uint32_t *vals, const uint32_t *offset, uint64_t n,
                           const uint32_t *start, uint32_t nb, uint64_t *buf_k, uint32_t *buf_v, uint64_t buf_len);
/* bucket_sort_device (src/pygpuhash.py:173-258): per-bucket rank sort into TK/TV[nb*520] */
int ec_hash_bucket_sort(const uint64_t *buf_k, const uint32_t *buf_v, uint64_t buf_len, const uint32_t *start,
                        const uint32_t *bucket_size, uint32_t nb, uint64_t *TK, uint32_t *TV);
/* debruijn_count_device (src/pydebruijn.py:15-178): lcount/ecount[size = 4V], updated in place */
int ec_db_counts(const uint64_t *lmer_keys, const uint32_t *lmer_values, uint64_t nl, uint32_t l, const uint64_t *TK,
                 const uint32_t *TV, const uint32_t *bucket_size, uint32_t nb, uint64_t size, uint32_t *lcount,
                 uint32_t *ecount);
/* setup_vertices_device (src/pydebruijn.py:181-324): ev[nk] updated in place */
int ec_db_vertices(const uint64_t *kmer_keys, uint64_t nk, const uint64_t *TK, const uint32_t *TV,
                   const uint32_t *bucket_size, uint32_t nb, const uint32_t *lcount, const uint32_t *lstart,
                   const uint32_t *ecount, const uint32_t *estart, void *ev);
/* setup_edges_device (src/pydebruijn.py:326-512): ee / l_out / e_out[E] updated in place */
int ec_db_edges(const uint64_t *lmer_keys, const uint32_t *lmer_values, const uint32_t *lmer_offsets, uint64_t nl,
                uint32_t l, const uint64_t *TK, const uint32_t *TV, const uint32_t *bucket_size, uint32_t nb,
                uint64_t nk, const uint32_t *lstart, const uint32_t *estart, unsigned flags, void *ee, uint32_t *l_out,
                uint32_t *e_out, uint64_t E);
/* assign_successor_device (src/pyeulertour.py:17-107): ee[e[ep+i]].s = l[lp+i] (in place) */
int ec_assign_successor(const void *ev, uint64_t vcount, const uint32_t *l, const uint32_t *e, void *ee, uint64_t E);
/* construct_successor_graphP1/P2_device (src/pyeulertour.py:109-216): Vertex{eid, s, pred} */
int ec_successor_graph(const void *ee, uint64_t E, void *vertices);
/* readLmersKmersCuda (src/eulercuda.py:73-179) host dedup, on the device: F / RC l-mer codes of
 * the concatenated buffer (L = lmerLength), distinct nonzero l-mers in first-occurrence order of
 * the stream F[0], R[0], F[1], ... with their counts, the number of zero ("empty") l-mers, and
 * the distinct (L-1)-mers of pF, sF, pR, sR per position in first-occurrence order.
 * Capacities: lmer_keys / lmer_values 2B, kmer_keys 4B; B < 2^30. */
int ec_read_lmers_kmers(const uint8_t *buf, uint64_t B, uint32_t L, uint64_t *lmer_keys, uint32_t *lmer_values,
                        uint64_t *n_lmers, uint64_t *lmer_empty, uint64_t *kmer_keys, uint64_t *n_kmers);
/* generatePartialContig (src/eulercuda.py:328-402) walk, on the device: every successor path
 * from its head (in head order), then every cycle from its smallest edge; contig c =
 * chars[coff[c] .. coff[c+1]) = getString(l-1, vid) of each edge's v1, then of the last edge's
 * v2.  Needs an injective successor map (EC_ERR_ARG otherwise).  Capacities: chars
 * 2E(l-1), coff E+1. */
int ec_partial_contigs(const void *ev, uint64_t vcount, const void *ee, uint64_t E, uint32_t l, char *chars,
                       uint64_t *coff, uint64_t *n_contigs, uint64_t *n_chars);

/* ---- step-level drop-ins of C1 and T3 (round 5) ------------------------------------------
 * One Shiloach-Vishkin step kernel of find_component_device (src/pycomponent.py:16-665) over
 * tid < length, in place on the caller's uint32 host arrays: step 0 componentStepInit (:34),
 * 1 / 2 ShortCuttingP1 / P2 (:87, :148), 3 / 4 StepTwoP1 / P2 (:212, :301), 5 / 6 StepThreeP1 /
 * P2 (:394, :474), 7 / 8 StepFourP1 / P2 (:548, :595), 9 StepFive (:638, sets *sptemp = 1).
 * Arrays a step does not touch may be null.  Replaces component_step_init ..
 * component_step5 (src/pycomponent.py:16, 66, 126, 187, 277, 369, 450, 529, 576, 625). */
int ec_component_step(int step, const void *vertices, uint32_t *prevD, uint32_t *D, uint32_t *Q, uint32_t *t1,
                      uint32_t *val1, uint32_t *t2, uint32_t *val2, uint32_t *sptemp, uint64_t length, uint32_t s);
/* calculate_circuit_graph_vertex_data_device (src/pyeulertour.py:219): C[D[i]] = 1, i < length
 * (EC_ERR_ARG if a label is >= ncount) */
int ec_cg_vertex_data(const uint32_t *D, uint64_t length, uint32_t *C, uint64_t ncount);
/* construct_circuit_Graph_vertex (src/pyeulertour.py:268): cv[offset[i]] = i where C[i] != 0 */
int ec_cg_vertices(const uint32_t *C, const uint32_t *offset, uint64_t ecount, uint32_t *cv, uint64_t ncv);
/* calculate_circuit_graph_edge_data (src/pyeulertour.py:307; cedge null: cedge_count[c] += the
 * circuit-graph edges of smaller end c) and assign_circuit_graph_edge_data (:393; cedge given:
 * the r-th edge of group c in sequential thread order at cedge[cedge_offset[c] + cedge_count[c]
 * - 1 - r], ceid untouched, cedge_count read only).  map = cg_offset (circuit label -> index). */
int ec_cg_edges_step(const void *ev, uint64_t vcount, const uint32_t *e, const uint32_t *D, const uint32_t *map,
                     uint64_t nmap, uint64_t ecount, const uint32_t *cedge_offset, uint32_t *cedge_count,
                     uint64_t ngroups, void *cedge, uint64_t cecount);

/* ---- native read ingest -----------------------------------------------
 * FASTA / FASTQ file -> packed bases + uint64 offsets (the CSR layout ec_assemble_* takes).
 * EC_FASTA_RECORDS: one read per '>' record, lines stripped and joined (SeqIO parse of
 *   tests/referenceAssembler.py:28; src/fastareader/parse_fasta.py:32-45; src/readTest.c:9-50);
 * EC_FASTA_LINES: one read per non-header line, stripped (read_fasta, src/eulercuda.py:437-445);
 * EC_FASTQ: line 1 of every 4-line record (read_fastq, src/eulercuda.py:43-55; a trailing '\r'
 *   is dropped).  threads <= 0: up to 16 host threads. */
#define EC_FASTA_RECORDS 0
#define EC_FASTA_LINES 1
#define EC_FASTQ 2
typedef struct ec_reads ec_reads;
int ec_reads_load(const char *path, int format, int threads, ec_reads **out);
uint64_t ec_reads_count(const ec_reads *r);
uint64_t ec_reads_bases(const ec_reads *r);
/* bases held by reads [first, first+count) (0 for a bad range) */
uint64_t ec_reads_span(const ec_reads *r, uint64_t first, uint64_t count);
/* copy reads [first, first+count): their bases and count+1 offsets rebased to 0 */
int ec_reads_copy(const ec_reads *r, uint64_t first, uint64_t count, uint8_t *bases, uint64_t *offsets);
void ec_reads_free(ec_reads *r);
/* ec_reads_free keeps one page-locked code buffer for the next EC_READS_PACKED load; this
 * releases it (teardown). */
void ec_reads_release_pool(void);
/* format | EC_READS_PACKED: ec_reads_load writes the bases straight as 2-bit codes (4 a byte, the
 * layout of ec_assemble_packed_host) into page-locked memory plus the bytes other than A/C/G/T as
 * (position, byte) exceptions -- no ASCII copy, no separate ec_pack_reads pass; read_len = the
 * common read length (0 if the lengths differ; then the offsets travel too) */
#define EC_READS_PACKED 0x100
int ec_reads_packed_info(const ec_reads *r, uint64_t *nbases, uint32_t *read_len, uint64_t *n_exc);
int ec_reads_packed_copy(const ec_reads *r, uint8_t *codes, uint64_t *exc_pos, uint8_t *exc_byte);
/* ec_assemble_packed_host on a packed read set (FASTA / FASTQ file -> contigs in two calls) */
int ec_assemble_packed_reads(ec_session *s, const ec_reads *r, int k, int limit, unsigned flags);
/* a packed read set as a staged batch (ec_stage_packed_host; r must outlive its assembly) */
int ec_stage_packed_reads(ec_session *s, const ec_reads *r);

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

/* count the shard (global read ids start at read_base, read_base + nreads <= 2^32); keeps
 * every distinct k-mer.  The count runs on shard-relative read ids (every shard qualifies
 * for the same count path); ec_export_by_owner writes global first events. */
int ec_count_shard(ec_session *s, const uint8_t *d_reads, const uint64_t *d_offsets, uint64_t nreads,
                   uint64_t read_base, int k, unsigned flags);
/* number of dense k-mer records the session holds (after ec_count_shard / ec_merge_owned) */
uint64_t ec_dense_count(ec_session *s);
/* pack the held records owner-major into d_out (ec_kmer_record[ec_dense_count]); owner_counts
 * (host, nowners <= 256) receives the records per owner.  d_out = NULL: counts only.
 * Owner of a canonical key: for 21 <= k <= 32 the range of its minimizer ((minimizer * nowners)
 * >> 32, the merge / load bucket key), else a 64-bit hash of the key (shard.h OwnerFn). */
int ec_export_by_owner(ec_session *s, int nowners, void *d_out, uint64_t *owner_counts);
/* the same with compact = 1 (round 5): where this shard's events fit, 20-B records (28 B for
 * k > 32: key, count, the two first events shard-relative as (read << *lf_bits) | position)
 * instead of 32 / 48 B, *lf_bits >= 0; else full records with global events, *lf_bits = -1.
 * d_out is sized for full records either way.  The receiver merges with ec_merge_owned_from. */
int ec_export_by_owner_ex(ec_session *s, int nowners, void *d_out, uint64_t *owner_counts, int compact,
                          int *lf_bits);
int ec_compact_record_bytes(int k);
/* ec_merge_owned on what nsrc ranks sent (source q: src_bytes[q] bytes, its global read base
 * and its records' lf_bits from ec_export_by_owner_ex; the sources in rank order) */
int ec_merge_owned_from(ec_session *s, const void *d_records, int nsrc, const uint64_t *src_bytes,
                        const int64_t *src_read_base, const int32_t *src_lf_bits, int k, int limit, unsigned flags);
/* owner rule of ec_export_by_owner: 0 (default) = the minimizer's range for 21 <= k <= 32, else a
 * key hash; 1 = the key hash always (distributed.py switches every rank to it when the job's
 * minimizer-range counts, all-reduced, show one owner past twice the mean -- low-complexity
 * input).  A counts-only call (d_out = NULL) followed by the scatter call reuses the owner ids. */
int ec_session_set_owner_rule(ec_session *s, int rule);
/* owner side: aggregate received records, keep count > limit */
int ec_merge_owned(ec_session *s, const void *d_records, uint64_t n, int k, int limit, unsigned flags);
/* copy the held records to d_out (after ec_count_shard with global first events, as the export) */
int ec_export_dense(ec_session *s, void *d_out);
/* ec_merge_owned + ec_export_dense in one call (no host round trip between them); d_out holds
 * up to n records, ec_dense_count gives how many were written */
int ec_merge_owned_export(ec_session *s, const void *d_records, uint64_t n, int k, int limit, unsigned flags,
                          void *d_out);
/* all_contigs(d, k) (referenceAssembler.py:79-111) on a caller's dict: n entries of k
 * characters (ACGT) in dict order with their counts; the dict must hold every k-mer together
 * with its twin, as build() returns it.  Results via ec_copy_contigs / ec_copy_links. */
int ec_assemble_from_kmers(ec_session *s, const char *kmers, const uint32_t *counts, uint64_t n, int k,
                           unsigned flags);
/* bytes per exchange record for node length k: 32 (ec_kmer_record, k <= 32) or 48
 * (ec_kmer_record_wide: uint64 lo, hi; uint32 count, pad; uint64 first_canon, first_twin, pad) */
int ec_record_bytes(int k);
/* graph phase (links .. GFA) on a complete solid set; results via ec_copy_* */
int ec_assemble_from_solid(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags);

/* partitioned graph phase (any k; records of ec_record_bytes(k)), the multi-GPU form of ec_assemble_from_solid: every rank
 * loads the same all-gathered solid set (dense ids = position among the non-filler records,
 * so identical on every rank; ec_dense_count = U), computes the successor links of its own
 * canonical ids [lo, hi) (d_succ receives 2(hi-lo) uint32 oriented-node successors, node
 * 2u+o, NONE = 0xFFFFFFFF), and after the caller's all-gather of those parts finishes the
 * graph phase on the complete successor array (uint32[2U], device) -- get_contig_forward:59-77
 * links, then ranking .. GFA as ec_assemble_from_solid; results via ec_copy_*. */
int ec_graph_load(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags);
int ec_graph_links_part(ec_session *s, uint64_t lo, uint64_t hi, uint32_t *d_succ);
/* ec_graph_load + ec_graph_links_part in one call (no host round trip between them) */
int ec_graph_load_links(ec_session *s, const void *d_records, uint64_t n, int k, unsigned flags, uint64_t lo,
                        uint64_t hi, uint32_t *d_succ);
int ec_graph_finish(ec_session *s, const uint32_t *d_succ, unsigned flags);

/* JUNCTION-PARTITIONED graph (round 5, csrc/junction.h): no rank holds the job's solid set.
 * After ec_merge_owned (this rank's owner segment, Ur keys):
 *   a. ec_graph_place: the segment placed at global canonical ids [lo, lo + Ur) of U (lo = the
 *      earlier ranks' segment sizes), its palindromes counted into *n_pal, and its (k-1)-mer
 *      junction records (ec_junction_record_bytes(k): 16 / 24 B, up to 4 Ur) written into d_jrecs
 *      grouped by the junction's owner (the keys' owner rule), owner_counts[r] records for rank r;
 *   b. (all-to-all-v of the records) ec_graph_join on everything this rank received (n records):
 *      the get_contig_forward links (referenceAssembler.py:59-73) of the junctions it owns --
 *      links of its own nodes kept, the others into d_links (ec_link_record_bytes() = 8 B, up
 *      to n) grouped by the node's rank, owner_counts[r] for rank r; seg_lo: the nowners + 1
 *      canonical id bounds of the segments (seg_lo[nowners] = U);
 *   c. (all-to-all-v of the link records) ec_graph_links_apply: the received links of its nodes.
 * The segment's successors are then in the session: ec_graph_chains_part takes d_succ = NULL.
 * Replaces the all-gather + ec_graph_load_links of the solid set (north_star: "redistributes
 * k-mers by hash prefix before each GPU builds its local graph partition"). */
int ec_graph_place(ec_session *s, uint64_t lo, uint64_t U, int nowners, void *d_jrecs, uint64_t *owner_counts,
                   uint64_t *n_pal);
int ec_graph_join(ec_session *s, const void *d_jrecs, uint64_t n, int nowners, const uint64_t *seg_lo, void *d_links,
                  uint64_t *owner_counts);
int ec_graph_links_apply(ec_session *s, const void *d_links, uint64_t n);
int ec_junction_record_bytes(int k);
int ec_link_record_bytes(void);

/* partitioned FINISH (round 4): instead of all-gathering the successor parts and ranking /
 * emitting the whole set on every rank (ec_graph_finish), each rank ranks and emits its own
 * segment [lo, hi) (a placed segment, or one of a loaded set) (csrc/rank_tile.h):
 *   1. ec_graph_chains_part: its successors' chains ranked in LDS tiles (d_succ: the segment's
 *      successors, or NULL for a placed segment, which holds them); its chains as super
 *      records (ec_super_record_bytes() = 32 B, up to 2(hi-lo)) into d_super, *n_super;
 *   2. ec_graph_rank_supers: every rank, on ALL super records (all-gathered, rank order) -- the
 *      order (n of them): the chains' list ranking (weighted ruling set);
 *   3. ec_graph_starts_part: its nodes' path keys / ranks, its contig starts as start records
 *      (ec_start_record_bytes() = 48 B, up to 2(hi-lo)) into d_starts, *n_starts (have_supers:
 *      the job had any super records);
 *   4. ec_graph_layout: every rank, on ALL start records (any order, n): contig order by first
 *      event, *n_chars = the job's contig characters;
 *      ec_graph_emit_part: its nodes' characters at their global positions into d_chars
 *      (n_chars bytes, zeroed by the caller) and the k-mer codes of the contigs' first / last
 *      nodes it holds into d_ends (2 * contigs codes of ec_end_record_bytes(k) = 8 / 16 B,
 *      zeroed) -- summed over the ranks they give every byte and end exactly once;
 *   5. ec_graph_collect (one rank): the summed characters / end codes -> GFA links
 *      (all_contigs:90-109, from the end codes alone) and the results (ec_copy_*,
 *      ec_get_stats; n_dict = 2 U - n_pal, n_pal = the job's palindromic solid k-mers). */
int ec_graph_chains_part(ec_session *s, uint64_t lo, uint64_t hi, const uint32_t *d_succ, void *d_super,
                         uint64_t *n_super);
int ec_graph_rank_supers(ec_session *s, const void *d_supers, uint64_t n);
int ec_graph_starts_part(ec_session *s, int have_supers, void *d_starts, uint64_t *n_starts);
int ec_graph_layout(ec_session *s, const void *d_starts, uint64_t n, uint64_t *n_chars);
int ec_graph_emit_part(ec_session *s, char *d_chars, void *d_ends);
int ec_graph_collect(ec_session *s, const char *d_chars, const void *d_ends, uint64_t n_pal);
/* The same emission and collection without job-sized buffers (round 6; distributed.py uses these
 * with engines that have them): ec_graph_emit_runs emits this rank's characters and contig ends
 * and sizes its transfer record -- the runs of consecutive character positions it wrote, their
 * characters, the ends it holds -- into *nbytes; ec_graph_copy_runs writes the record into d_out
 * (nbytes, 8-byte aligned; stream-ordered).  The records of all ranks are gathered (concatenated
 * in rank order, src_bytes[r] each) to the collecting rank, whose ec_graph_collect_runs scatters
 * them into the job's characters and ends and finishes as ec_graph_collect. */
int ec_graph_emit_runs(ec_session *s, uint64_t *nbytes);
/* Exact-size outputs (round 6): ec_graph_place, ec_graph_chains_part and ec_graph_starts_part
 * called with a NULL output (d_jrecs / d_super / d_starts) count their records only (the counts
 * returned as above) and hold them; the matching copy, before any other step of the session,
 * writes them into a buffer of exactly that many records -- instead of the upper bounds (4 Ur
 * junction records, 2 (hi - lo) super / start records: ~50 GB at config 5's per-rank size).
 * ec_graph_chains_part on a placed segment keeps its tile records in the junction-record buffer
 * ec_graph_place filled, so place records still held then are dropped (ec_graph_place_copy
 * returns EC_ERR_STATE). */
int ec_graph_place_copy(ec_session *s, void *d_jrecs);
int ec_graph_chains_copy(ec_session *s, void *d_super);
int ec_graph_starts_copy(ec_session *s, void *d_starts);
int ec_graph_copy_runs(ec_session *s, void *d_out);
int ec_graph_collect_runs(ec_session *s, const void *d_in, int nsrc, const uint64_t *src_bytes, uint64_t n_pal);
int ec_end_record_bytes(int k);
int ec_super_record_bytes(void);
int ec_start_record_bytes(void);

#ifdef __cplusplus
}
#endif
#endif /* EULERHIP_H */
