// junction.h -- the multi-GPU graph partition without a global solid set (round 5).
//
// Up to round 4 every rank all-gathered the job's solid set (148 MB at config 4), loaded it
// (0.4 ms) and probed it for the links of its own owner segment.  Here a rank keeps only its own
// segment -- the k-mers its owner merge produced, placed at their global dense ids -- and the
// successor links come out of the (k - 1)-mer half-edge join of join_w.h run ACROSS ranks:
//
//   ec_graph_place      the segment's dense arrays moved to global ids [lo, lo + Ur); every
//                       canonical key emits its two junction records (suffix / prefix (k-1)-mer,
//                       canonicalised, tagged with the oriented global node id, side and the
//                       node's palindrome flag) routed to the JUNCTION's owner.  With minimizer
//                       owners a junction's minimizer is its k-mers' minimizer for (w-1)/w of
//                       them, so nearly all records stay on their rank.
//   (all-to-all-v of the records)
//   ec_graph_join       per final bucket (hash of the junction) an LDS table collects one node
//                       id per side; a junction with one id on each side and y != twin(x) gives
//                       succ[x] = y and succ[twin y] = twin x -- written locally when the node is
//                       in this rank's segment, else as an 8-B link record for its owner
//   (all-to-all-v of the link records)
//   ec_graph_links_apply
//
// The result is the segment part of the successor array ec_graph_links_part computed on the
// loaded set, without loading it (get_contig_forward's rule, referenceAssembler.py:59-73).
#pragma once
#include "join_w.h"
#include "shard.h"

namespace ec {

// junction records on the wire: RecJ64 (k <= 32: 16 B) / RecJ (k > 32: 24 B), pad = the node's
// palindrome flag (twin(x) = x for a palindromic k-mer, x ^ 1 otherwise)
__device__ inline K128 jkey(const RecJ64 &r) { return K128{r.key, 0ull}; }
__device__ inline K128 jkey(const RecJ &r) { return K128{r.lo, r.hi}; }
__device__ inline uint64_t jhash(const RecJ64 &r) { return mix64(r.key); }
__device__ inline uint64_t jhash(const RecJ &r) { return mix128(K128{r.lo, r.hi}); }

// minimizer of a canonical j-mer held in a K128 (j <= 62; twin_j handles j <= 32)
__device__ inline uint32_t minimizer_of_wj(const K128 &c, int j) {
    const K128 tc = twin_j(c, j);
    const int w = j - SK_M + 1;
    uint32_t v = 0xFFFFFFFFu;
    for (int p = 0; p < w; p++) {
        const uint32_t f = bits30_128(c, 2 * (j - SK_M - p)), r = bits30_128(tc, 2 * p);
        const uint32_t h = mmer_hash(f < r ? f : r);
        v = h < v ? h : v;
    }
    return min_remix_w(v);
}

// owner of a canonical junction (j = k - 1 bases) under the key owner rule: the range of its
// minimizer where keys use minimizer owners (own.sk / own.wk), else a hash
struct JOwnerFn {
    MinCfg mcj;  // sk_cfg(j) when own.sk
    int sk, wj;  // wj: j when own.wk
    __device__ inline unsigned int operator()(const RecJ64 &r, unsigned int n) const {
        return sk ? (unsigned int)(((uint64_t)minimizer_of(r.key, mcj) * n) >> 32) : owner_of(r.key, n);
    }
    __device__ inline unsigned int operator()(const RecJ &r, unsigned int n) const {
        const K128 o{r.lo, r.hi};
        return wj ? (unsigned int)(((uint64_t)minimizer_of_wj(o, wj) * n) >> 32) : owner_of(o, n);
    }
};

template <typename K> struct JRecOf;
template <> struct JRecOf<unsigned long long> { using R = RecJ64; };
template <> struct JRecOf<K128> { using R = RecJ; };

// the segment's junction records with their owners: slot 4 t + q of canonical key t (q = 0, 1:
// suffix / prefix records; 2, 3: the second records of a palindromic junction, else empty);
// owner NONE for empty slots.  Node ids are global: 2 (lo + t) + o.
template <typename K>
__global__ void __launch_bounds__(256) k_junction_emit(const K *dkey, const uint8_t *upal, unsigned int lo,
                                                       unsigned int Ur, int k, JOwnerFn own, unsigned int nowners,
                                                       typename JRecOf<K>::R *out, unsigned int *oid) {
    using R = typename JRecOf<K>::R;
    const int j = k - 1;
    const K mj = kmask_j(j, (K *)nullptr);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < Ur; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int g = lo + (unsigned int)t;
        R r1, r2, x1, x2;
        bool e1, e2;
        half_recs(dkey[g], g, j, mj, upal, r1, r2, e1, e2, x1, x2);
        const unsigned int pal = upal[g];
        r1.pad = r2.pad = x1.pad = x2.pad = pal;
        const uint64_t b = 4 * t;
        out[b] = r1;
        oid[b] = own(r1, nowners);
        out[b + 1] = r2;
        oid[b + 1] = own(r2, nowners);
        out[b + 2] = x1;
        oid[b + 2] = e1 ? own(x1, nowners) : NONE32;
        out[b + 3] = x2;
        oid[b + 3] = e2 ? own(x2, nowners) : NONE32;
    }
}

// empty record slots (owner NONE) -> bin nowners, past the owners' bins
__global__ void __launch_bounds__(256) k_none_to_bin(unsigned int *oid, uint64_t n, unsigned int nowners) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (oid[i] == NONE32) oid[i] = nowners;
}

// out[i] = in[perm[i]] for the first n of a permutation
template <typename R>
__global__ void __launch_bounds__(256) k_gather_recs(const R *in, const unsigned int *perm, uint64_t n, R *out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[perm[i]];
}

// join bucket of a record: top bt bits of the junction's hash
template <typename R>
__global__ void __launch_bounds__(256) k_junction_bucket(const R *recs, uint64_t n, int bt, unsigned int *bid) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        bid[i] = bt ? (unsigned int)(jhash(recs[i]) >> (64 - bt)) : 0u;
}

// owner rank of a global canonical id (seg_lo: nowners + 1 ascending bounds)
__device__ inline unsigned int seg_owner(const unsigned long long *seg_lo, unsigned int nowners, unsigned int c) {
    unsigned int a = 0, b = nowners;  // seg_lo[a] <= c < seg_lo[b]
    while (b - a > 1) {
        const unsigned int m = (a + b) >> 1;
        if ((unsigned long long)c >= seg_lo[m]) a = m;
        else b = m;
    }
    return a;
}

// link record for another rank's node: succ[node] = value
struct LinkRec {
    unsigned int node, value;
};
static_assert(sizeof(LinkRec) == 8, "link record layout");

// The join across ranks: per bucket b the records perm[bstart[b] .. bstart[b + 1]) grouped by
// junction in an LDS table (as k_half_join: two CASes on the key's 63-bit halves, one id per
// side whose MANY bit marks a second distinct id; ids carry the palindrome flag above bit 32).
// Links of nodes in [n0, n1) go to succ, others to the link outbox (wave-aggregated append).
//
// More junctions than 2^14 buckets of tables hold (a rank past ~4.7 * 10^7 junctions): every
// bucket is split again by the next sbits hash bits into 2^sbits sub-buckets, which the
// workgroup joins one after the other in its table (its records read once per sub-bucket; the
// bucket sort stays at <= 2^14 bins, the LDS histogram's limit).  claim: slots a table may
// claim (SLOTS - 1; smaller only to test the overflow retries).
template <int SLOTS, int NT, typename R>
__global__ void __launch_bounds__(NT) k_junction_join(const R *recs, const unsigned int *perm,
                                                      const unsigned long long *bstart, unsigned int n0,
                                                      unsigned int n1, unsigned int *succ, LinkRec *outbox,
                                                      unsigned int *nout, unsigned int outcap, unsigned int *overflow,
                                                      int bt, int sbits, unsigned int claim) {
    constexpr unsigned long long EMPTY = ~0ull, MANY = 1ull << 62;
    // 4 SLOTS x 8 B of tables: 64 KB at 2048 slots, 128 KB at 4096 -- gfx950's 160 KB of LDS
    // per workgroup (earlier CDNA parts allow 64 KB: the 4096-slot table needs MI355X)
    static_assert(4 * SLOTS * 8 + 64 <= 160 * 1024, "junction tables exceed gfx950's LDS per workgroup");
    __shared__ unsigned long long w1[SLOTS], w2[SLOTS];
    __shared__ unsigned long long ids[2][SLOTS];
    __shared__ unsigned int s_over[2];
    __shared__ unsigned int s_cnt, s_base;
    const unsigned int b = blockIdx.x;
    const uint64_t r0 = bstart[b], r1 = bstart[b + 1];
    const unsigned int nsub = 1u << sbits;
    for (unsigned int sub = 0; sub < nsub; sub++) {
    for (int i = threadIdx.x; i < SLOTS; i += NT) {
        w1[i] = 0;
        w2[i] = 0;
        ids[0][i] = EMPTY;
        ids[1][i] = EMPTY;
    }
    if (threadIdx.x == 0) {
        s_over[0] = 0;
        s_over[1] = 0;
    }
    __syncthreads();
    for (uint64_t base = r0; base < r1; base += NT) {
        const uint64_t i = base + threadIdx.x;
        bool valid = i < r1;
        R r{};
        if (valid) r = recs[perm[i]];
        if (sbits && valid) valid = (unsigned int)((jhash(r) << bt) >> (64 - sbits)) == sub;
        const K128 o = jkey(r);
        const unsigned long long a1 = wide_w1(o), a2 = wide_w2(o);
        unsigned int slot = (unsigned int)(((uint64_t)(uint32_t)jhash(r) * SLOTS) >> 32);
        unsigned long long a = 0, bw = 0;
        bool miss = valid;
        if (valid) {
            a = w1[slot];
            bw = w2[slot];
            miss = !(a == a1 && bw == a2);
        }
#pragma unroll 1
        while (__any(miss)) {
            if (miss) {
                if (a == 0) {
                    if (atomicAdd(&s_over[1], 1u) >= claim) {
                        s_over[0] = 1;
                        a = a1;
                        bw = a2;
                    } else {
                        a = atomicCAS(&w1[slot], 0ull, a1);
                        if (a == 0) a = a1;
                        else atomicSub(&s_over[1], 1u);
                    }
                }
                if (a == a1 && bw != a2) {
                    bw = w2[slot];
                    if (bw == 0) {
                        bw = atomicCAS(&w2[slot], 0ull, a2);
                        if (bw == 0) bw = a2;
                    }
                }
                if (!(a == a1 && bw == a2)) {
                    slot = slot + 1 == SLOTS ? 0u : slot + 1;
                    a = w1[slot];
                    bw = w2[slot];
                }
                miss = !(a == a1 && bw == a2);
            }
        }
        if (valid) {
            const unsigned int side = r.tag >> 31, id = r.tag & 0x7FFFFFFFu;
            const unsigned long long v = ((unsigned long long)(r.pad & 1u) << 32) | id;
            const unsigned long long old = atomicCAS(&ids[side][slot], EMPTY, v);
            if (old != EMPTY && (unsigned int)old != id) atomicOr(&ids[side][slot], MANY);
        }
    }
    __syncthreads();
    if (s_over[0]) {  // (uniform: the host retries with finer buckets)
        if (threadIdx.x == 0) atomicOr(overflow, 1u);
        return;
    }
    // links: local ones written at once; the other ranks' into the outbox at one global
    // reservation per workgroup (a counter hit by every wave serialises at the memory side: ~60 K
    // appends a rank took 0.46 ms)
    constexpr int PER = (SLOTS + NT - 1) / NT;
    unsigned int rt[2 * PER], rv[2 * PER], nr = 0;  // (static indices: registers, no scratch)
    bool rf[2 * PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int i = threadIdx.x + q * NT;
        rf[2 * q] = rf[2 * q + 1] = false;
        if (i >= SLOTS) continue;
        const unsigned long long ex = ids[0][i], ey = ids[1][i];
        if (ex == EMPTY || ey == EMPTY || ((ex | ey) & MANY)) continue;
        const unsigned int x = (unsigned int)ex, y = (unsigned int)ey;
        const unsigned int tx = (ex >> 32) ? x : (x ^ 1u), ty = (ey >> 32) ? y : (y ^ 1u);
        if (y == tx) continue;
        rt[2 * q] = x, rv[2 * q] = y, rf[2 * q] = !(x >= n0 && x < n1);
        rt[2 * q + 1] = ty, rv[2 * q + 1] = tx, rf[2 * q + 1] = !(ty >= n0 && ty < n1);
        if (!rf[2 * q]) succ[x] = y;
        if (!rf[2 * q + 1]) succ[ty] = tx;
        nr += rf[2 * q] + rf[2 * q + 1];
    }
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const unsigned int my = nr ? atomicAdd(&s_cnt, nr) : 0u;
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(nout, s_cnt) : 0u;
    __syncthreads();
    unsigned int p = s_base + my;
#pragma unroll
    for (int j = 0; j < 2 * PER; j++) {
        if (!rf[j]) continue;
        if (p < outcap) outbox[p] = LinkRec{rt[j], rv[j]};
        else atomicOr(overflow, 2u);
        p++;
    }
    __syncthreads();  // (the next sub-bucket clears the tables)
    }
}

// destination rank of every outbox link record (bin nowners past the count: none)
__global__ void __launch_bounds__(256) k_link_dest(const LinkRec *out, const unsigned int *nout, unsigned int cap,
                                                   const unsigned long long *seg_lo, unsigned int nowners,
                                                   unsigned int *bid) {
    const unsigned int n = min(*nout, cap);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x)
        bid[i] = i < n ? seg_owner(seg_lo, nowners, out[i].node >> 1) : nowners;
}

// received link records of this rank's nodes
__global__ void __launch_bounds__(256) k_links_apply(const LinkRec *in, uint64_t n, unsigned int n0, unsigned int n1,
                                                     unsigned int *succ, unsigned int *bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const LinkRec r = in[i];
        if (r.node >= n0 && r.node < n1) succ[r.node] = r.value;
        else atomicOr(bad, 1u);
    }
}

// ---- GFA links from contig-end codes (the partitioned finish's rank 0 holds no global set) ----
// ends[i] / ends[nc + i]: codes of contig i's first / last oriented k-mer (each written by the
// rank that emitted that node).  A table keyed by canonical code holds, per orientation, the
// contig whose head it is and the contig whose twin-tail it is: headOf / tailOf of k_emit for
// the only nodes that have them, so all_contigs:90-109's lookups need nothing else.
struct EndSlot64 {
    unsigned long long key;
    unsigned int hd[2], tl[2];  // [orientation]: head of / twin-tail of contig
};
struct EndSlotW {
    unsigned long long w1, w2;
    unsigned int hd[2], tl[2];
};
template <typename K> struct EndSlotOf;
template <> struct EndSlotOf<unsigned long long> { using T = EndSlot64; };
template <> struct EndSlotOf<K128> { using T = EndSlotW; };

__global__ void __launch_bounds__(256) k_end_clear64(EndSlot64 *t, uint64_t cap) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        t[i].key = EMPTY_KEY;
        t[i].hd[0] = t[i].hd[1] = t[i].tl[0] = t[i].tl[1] = NONE32;
    }
}
__global__ void __launch_bounds__(256) k_end_clearW(EndSlotW *t, uint64_t cap) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        t[i].w1 = t[i].w2 = 0;
        t[i].hd[0] = t[i].hd[1] = t[i].tl[0] = t[i].tl[1] = NONE32;
    }
}
// find-or-insert of canonical code c (capmask + 1 slots, > 2 x the entries: no overflow)
__device__ inline EndSlot64 *end_slot(EndSlot64 *t, uint64_t capmask, unsigned long long c, bool ins) {
    uint64_t h = mix64(c) & capmask;
    for (;;) {
        unsigned long long cur = t[h].key;
        if (cur == EMPTY_KEY) {
            if (!ins) return nullptr;
            cur = atomicCAS(&t[h].key, EMPTY_KEY, c);
            if (cur == EMPTY_KEY) return t + h;
        }
        if (cur == c) return t + h;
        h = (h + 1) & capmask;
    }
}
__device__ inline EndSlotW *end_slot(EndSlotW *t, uint64_t capmask, const K128 &c, bool ins) {
    const unsigned long long w1 = wide_w1(c), w2 = wide_w2(c);
    uint64_t h = mix128(c) & capmask;
    for (;;) {
        EndSlotW *sl = t + h;
        unsigned long long a = sl->w1;
        if (a == 0) {
            if (!ins) return nullptr;
            a = atomicCAS(&sl->w1, 0ull, w1);
            if (a == 0) a = w1;
        }
        if (a == w1) {
            unsigned long long b = sl->w2;
            if (b == 0) {
                if (!ins) return nullptr;  // (a claim in flight: only during the insert pass)
                b = atomicCAS(&sl->w2, 0ull, w2);
                if (b == 0) b = w2;
            }
            if (b == w2) return sl;
        }
        h = (h + 1) & capmask;
    }
}

template <typename Ops>
__global__ void __launch_bounds__(256) k_end_insert(const typename Ops::K *ends, unsigned int nc, int k,
                                                    typename EndSlotOf<typename Ops::K>::T *t, uint64_t capmask) {
    using K = typename Ops::K;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        const K f = ends[i], tl = Ops::twin(ends[nc + i], k);  // head node; the last node's twin
        {
            const K tf = Ops::twin(f, k), cf = f < tf ? f : tf;
            atomicMin(&end_slot(t, capmask, cf, true)->hd[f == cf ? 0 : 1], (unsigned int)i);
        }
        {
            const K tt = Ops::twin(tl, k), ct = tl < tt ? tl : tt;
            atomicMin(&end_slot(t, capmask, ct, true)->tl[tl == ct ? 0 : 1], (unsigned int)i);
        }
    }
}

// k_gfa on codes: for y in fw(last k-mer): heads[y] then tails[y]; for z in fw(twin(first)):
// heads[z] then tails[z] (all_contigs:90-109)
template <typename Ops>
__global__ void __launch_bounds__(256) k_gfa_codes(const typename Ops::K *ends, unsigned int nc, int k,
                                                   const typename EndSlotOf<typename Ops::K>::T *t, uint64_t capmask,
                                                   long long *lk, unsigned int *lcnt) {
    using K = typename Ops::K;
    using T = typename EndSlotOf<K>::T;
    const K mask = Ops::mask(k);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        for (int side = 0; side < 2; side++) {
            const K xs = side == 0 ? ends[nc + i] : Ops::twin(ends[i], k);
            unsigned int n = 0;
            long long *o = lk + (i * 2 + side) * 8;
            for (uint32_t b = 0; b < 4; b++) {
                const K y = Ops::push(xs, b, mask);
                const K ty = Ops::twin(y, k);
                const K cy = y < ty ? y : ty;
                const T *sl = end_slot(const_cast<T *>(t), capmask, cy, false);
                if (!sl) continue;
                const int oy = y == cy ? 0 : 1;
                if (sl->hd[oy] != NONE32) o[n++] = 2ll * sl->hd[oy];
                if (sl->tl[oy] != NONE32) o[n++] = 2ll * sl->tl[oy] + 1;
            }
            lcnt[i * 2 + side] = n;
        }
    }
}

// k_emit's contig ends as codes (ends pre-zeroed; this rank writes the ends of its own nodes)
template <typename Ops>
__global__ void __launch_bounds__(256) k_ends_codes(const unsigned int *cfirst, const unsigned int *clast, unsigned int nc,
                                                    const typename Ops::K *dkey, int k, typename Ops::K *ends) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        if (cfirst[i] != NONE32) ends[i] = node_code<Ops>(dkey, cfirst[i], k);
        if (clast[i] != NONE32) ends[nc + i] = node_code<Ops>(dkey, clast[i], k);
    }
}

// ---- the partitioned finish's transfer to the collecting rank (round 6) ---------------------
// Up to round 5 every rank emitted into a zeroed job-sized character buffer and a job-sized end
// table, and one reduce-sum brought both to rank 0 (config 5: ~2 * 10^8 B a rank).  Now a rank
// sends only what it wrote: runs of consecutive character positions (cut at RUN_CH-position
// chunks) and the contig ends it holds, one transfer record a rank, gathered to rank 0:
//   u64 header[4] = {runs, characters, ends, 0}
//   u64 start[runs]   job position of each run's first character
//   u64 coff[runs]    offset of its first character in chars (its length: the next one's - it)
//   u8  chars[characters], padded to 8
//   EndRec ends[ends] (idx = contig for its first k-mer, nc + contig for its last)
constexpr unsigned int RUN_CH = 4096;  // positions a compaction workgroup scans (16 a thread)
constexpr unsigned int RUN_NT = RUN_CH / 16;
template <typename K>
struct EndRec {
    unsigned int idx, pad;
    K code;
};
__host__ __device__ inline uint64_t run_rec_bytes(uint64_t runs, uint64_t chars, uint64_t ends, int kbytes) {
    return 32 + 16 * runs + ((chars + 7) & ~7ull) + ends * (8 + (uint64_t)kbytes);
}

// written (non-zero) bytes of a thread's 16 positions and the run starts among them (a run starts
// at a written byte whose predecessor is not written, or at the chunk's first position)
__device__ inline void run_masks(const uint8_t *chars, uint64_t n, uint64_t p, uint32_t *s_nz, uint32_t &nz,
                                 uint32_t &st) {
    nz = 0;
    if (p < n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(chars + p);  // (the buffer has 16 B of padding)
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t m = (((w[u] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w[u]) & 0x80808080u;  // byte != 0
            nz |= (((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u)) << (4 * u);
        }
        if (n - p < 16) nz &= (1u << (n - p)) - 1u;
    }
    s_nz[threadIdx.x] = nz;
    __syncthreads();
    const uint32_t prev = threadIdx.x ? (s_nz[threadIdx.x - 1] >> 15) & 1u : 0u;
    st = nz & ~((nz << 1) | prev) & 0xFFFFu;
}
// runs and characters of chunk blockIdx.x -> rc[chunk], cc[chunk]
__global__ void __launch_bounds__(RUN_NT) k_runs_count(const uint8_t *chars, uint64_t n, unsigned long long *rc,
                                                       unsigned long long *cc) {
    __shared__ uint32_t s_nz[RUN_NT];
    __shared__ unsigned int s_r[RUN_NT / 64], s_c[RUN_NT / 64];
    uint32_t nz, st;
    run_masks(chars, n, (uint64_t)blockIdx.x * RUN_CH + 16ull * threadIdx.x, s_nz, nz, st);
    unsigned int r = (unsigned int)__popc(st), c = (unsigned int)__popc(nz);
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o), c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) s_r[threadIdx.x >> 6] = r, s_c[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long R = 0, C = 0;
        for (unsigned int q = 0; q < RUN_NT / 64; q++) R += s_r[q], C += s_c[q];
        rc[blockIdx.x] = R;
        cc[blockIdx.x] = C;
    }
}
// the chunk's runs and characters at the scanned bases (rb, cb: exclusive scans of rc, cc)
__global__ void __launch_bounds__(RUN_NT) k_runs_write(const uint8_t *chars, uint64_t n, const unsigned long long *rb,
                                                       const unsigned long long *cb, unsigned long long *rstart,
                                                       unsigned long long *rcoff, uint8_t *rchars) {
    __shared__ uint32_t s_nz[RUN_NT];
    __shared__ unsigned int s_r[RUN_NT], s_c[RUN_NT];
    const uint64_t p = (uint64_t)blockIdx.x * RUN_CH + 16ull * threadIdx.x;
    uint32_t nz, st;
    run_masks(chars, n, p, s_nz, nz, st);
    const unsigned int r = (unsigned int)__popc(st), c = (unsigned int)__popc(nz);
    s_r[threadIdx.x] = r;
    s_c[threadIdx.x] = c;
    __syncthreads();
    for (unsigned int o = 1; o < RUN_NT; o <<= 1) {  // inclusive block scans
        const unsigned int ar = threadIdx.x >= o ? s_r[threadIdx.x - o] : 0u;
        const unsigned int ac = threadIdx.x >= o ? s_c[threadIdx.x - o] : 0u;
        __syncthreads();
        s_r[threadIdx.x] += ar;
        s_c[threadIdx.x] += ac;
        __syncthreads();
    }
    unsigned long long ri = rb[blockIdx.x] + s_r[threadIdx.x] - r, ci = cb[blockIdx.x] + s_c[threadIdx.x] - c;
    for (int i = 0; i < 16; i++) {
        if (!((nz >> i) & 1u)) continue;
        if ((st >> i) & 1u) {
            rstart[ri] = p + i;
            rcoff[ri] = ci;
            ri++;
        }
        rchars[ci++] = chars[p + i];
    }
}
// the contig ends this rank emitted (cfirst / clast set) as EndRecs, appended
template <typename Ops>
__global__ void __launch_bounds__(256) k_ends_recs(const unsigned int *cfirst, const unsigned int *clast, unsigned int nc,
                                                   const typename Ops::K *dkey, int k,
                                                   EndRec<typename Ops::K> *out, unsigned int *nout) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        if (cfirst[i] != NONE32) {
            EndRec<typename Ops::K> e;
            e.idx = (unsigned int)i, e.pad = 0, e.code = node_code<Ops>(dkey, cfirst[i], k);
            out[atomicAdd(nout, 1u)] = e;
        }
        if (clast[i] != NONE32) {
            EndRec<typename Ops::K> e;
            e.idx = nc + (unsigned int)i, e.pad = 0, e.code = node_code<Ops>(dkey, clast[i], k);
            out[atomicAdd(nout, 1u)] = e;
        }
    }
}
__global__ void k_put_u64x4(unsigned long long *d, unsigned long long a, unsigned long long b, unsigned long long c,
                            unsigned long long e) {
    if (threadIdx.x == 0) d[0] = a, d[1] = b, d[2] = c, d[3] = e;
}
// collecting rank: a source's runs into the job's characters, its ends into the end table
__global__ void __launch_bounds__(256) k_runs_scatter(const unsigned long long *rstart, const unsigned long long *rcoff,
                                                      uint64_t nr, uint64_t nch, const uint8_t *rchars, uint8_t *chars,
                                                      uint64_t nchars, unsigned int *bad) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nr; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c0 = rcoff[r], c1 = r + 1 < nr ? rcoff[r + 1] : nch, p = rstart[r];
        if (c1 < c0 || c1 > nch || p + (c1 - c0) > nchars) {
            atomicOr(bad, 1u);
            continue;
        }
        for (uint64_t c = c0; c < c1; c++) chars[p + (c - c0)] = rchars[c];
    }
}
template <typename K>
__global__ void __launch_bounds__(256) k_ends_scatter(const EndRec<K> *in, uint64_t n, unsigned int nc2, K *ends,
                                                      unsigned int *bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const EndRec<K> e = in[i];
        if (e.idx < nc2) ends[e.idx] = e.code;
        else atomicOr(bad, 1u);
    }
}

}  // namespace ec
