// graph.h -- de Bruijn links, list ranking, contig starts/order, emission, GFA links.
#pragma once
#include "count_global.h"
#include "count_part.h"
#include "superkmer.h"
#include "wide.h"

namespace ec {

// canonical key -> dense solid id (NONE if absent or not solid).  Two layouts: the bucketed
// sub-tables written by k_bucket / k_bucket_sk (partitioned paths; the bucket of a key is the
// top bits of mix64(key), or of its minimizer on the super-k-mer path) or the single HBM table
// (general path).  Within a bucket the first probe slot is slot0(key), as in lds_insert.
struct SolidIndex {
    const Slot *table;
    uint64_t capmask;
    const SubSlot *sub;
    int bbits;
    unsigned int slots;  // sub-table slots per bucket (power of 2)
    int sk;              // buckets by minimizer (superkmer.h)
    const uint8_t *npb;  // k_bucket_filt layout: bucket b split into 2^npb[b] parts (hash bits 11..)
    int pmax;            // of a region of 2^pmax part tables
    MinCfg mc;
    int bijk = 0;        // count_v2.h 10-byte records (k): sub-tables keyed by bij_fwd(key), bucket = its top bits
    // (measured: a wave-uniform probe loop with 16-B key+id loads made k_neighbors 0.70 ->
    // 1.3 ms; the per-lane loop below lets the four neighbour lookups overlap)
    __device__ inline unsigned int find_in(uint64_t c, unsigned int h, uint64_t b) const {
        const SubSlot *r = sub + b * slots;
        unsigned int n = slots;
        if (npb) {
            n = slots >> pmax;
            r += ((h >> 11) & ((1u << npb[b]) - 1)) * n;
        }
        unsigned int slot = h & (n - 1);
        for (unsigned int probe = 0; probe < n; probe++) {
            const unsigned long long kk = r[slot].key;
            if (kk == c) return r[slot].id;
            if (kk == EMPTY_KEY) return NONE32;
            slot = (slot + 1) & (n - 1);
        }
        return NONE32;
    }
    // first probe slot in a bucket sub-table (k_bucket: mix64, k_bucket_sk: sk_slot top bits)
    __device__ inline unsigned int slot0(uint64_t c) const {
        return sk ? sk_slot(c) >> (32 - __builtin_ctz(slots)) : (unsigned int)mix64(c);
    }
    __device__ inline unsigned int find(uint64_t c) const {
        if (sub && bijk) {
            const uint64_t hc = bij_fwd(c, bijk, kmask64(bijk));  // slot: hc itself (Rec12PSource<., true>)
            return find_in(hc, (unsigned int)hc, bbits ? (hc >> (2 * bijk - bbits)) : 0);
        }
        if (sub) {
            const uint64_t h = mix64(c);
            const uint64_t b = sk ? sk_bucket_of(minimizer_of(c, mc), bbits) : (bbits ? (h >> (64 - bbits)) : 0);
            return find_in(c, slot0(c), b);
        }
        return lookup(table, capmask, c);
    }
    // successors of oriented k-mer xs (k-mers xs << 2 | b): on the super-k-mer path their
    // minimizers share the w - 1 m-mers of xs's last k - 1 bases.  txs = twin(xs): the reverse
    // complement of xs's m-mer p is txs's m-mer at offset p from the end (no per-m-mer reversal)
    struct Nb {
        uint32_t part;
    };
    __device__ inline Nb nb_begin(uint64_t xs, uint64_t txs) const {
        Nb nb{0xFFFFFFFFu};
        if (sub && sk)
            for (int p = 1; p < mc.w; p++) {
                const uint32_t f = (uint32_t)(xs >> (2 * (mc.k - mc.m - p))) & mc.mmask;
                const uint32_t r = (uint32_t)(txs >> (2 * p)) & mc.mmask;
                const uint32_t h = mmer_hash(f < r ? f : r);
                nb.part = h < nb.part ? h : nb.part;
            }
        return nb;
    }
    // successor y = xs << 2 | b, ty = twin(y), cy = canonical
    __device__ inline unsigned int find_nb(const Nb &nb, uint64_t y, uint64_t ty, uint64_t cy) const {
        if (sub && sk) {
            const uint32_t f = (uint32_t)y & mc.mmask, r = (uint32_t)(ty >> (2 * (mc.k - mc.m))) & mc.mmask;
            const uint32_t h = mmer_hash(f < r ? f : r);
            return find_in(cy, slot0(cy), sk_bucket_of(min_remix(h < nb.part ? h : nb.part), bbits));
        }
        return find(cy);
    }
};
// key algebra of the graph phase: 64-bit codes (k <= 32) or K128 (32 < k <= 63)
struct Ops64 {
    using K = unsigned long long;
    __device__ static inline K mask(int k) { return kmask64(k); }
    __device__ static inline K twin(const K &x, int k) { return twin64(x, k); }
    __device__ static inline K push(const K &x, uint32_t b, const K &m) { return ((x << 2) | b) & m; }
    // twin(push(x, b)) from tx = twin(x): the complement of b enters at the front
    __device__ static inline K twin_push(const K &tx, uint32_t b, int k) {
        return (tx >> 2) | ((K)(3u - b) << (2 * (k - 1)));
    }
    __device__ static inline uint32_t base(const K &x, int k, int i) { return (uint32_t)(x >> (2 * (k - 1 - i))) & 3u; }
    __device__ static inline uint32_t last(const K &x) { return (uint32_t)x & 3u; }
    __device__ static inline char chr(uint32_t b) { return "ACGT"[b]; }  // symbol code -> byte
};
struct OpsW {
    using K = K128;
    __device__ static inline K mask(int k) { return kmask128(k); }
    __device__ static inline K twin(const K &x, int k) { return twin128(x, k); }
    __device__ static inline K push(const K &x, uint32_t b, const K &m) { return push128(x, b, m); }
    __device__ static inline K twin_push(const K &tx, uint32_t b, int k) {  // 2(k-1) >= 64
        K r;
        r.lo = (tx.lo >> 2) | (tx.hi << 62);
        r.hi = (tx.hi >> 2) | ((unsigned long long)(3u - b) << (2 * (k - 1) - 64));
        return r;
    }
    __device__ static inline uint32_t base(const K &x, int k, int i) { return base_at128(x, k, i); }
    __device__ static inline uint32_t last(const K &x) { return (uint32_t)x.lo & 3u; }
    __device__ static inline char chr(uint32_t b) { return "ACGT"[b]; }
};

// canonical K128 key -> dense solid id in the wide table
// minimizer buckets of 128-bit keys (count_wide.h, round 4): a key's placement hash
__host__ __device__ inline uint32_t bits30_128(const K128 &x, int sh) {  // 0 <= sh <= 98
    const uint64_t v = sh >= 64 ? (x.hi >> (sh - 64)) : sh == 0 ? x.lo : ((x.lo >> sh) | (x.hi << (64 - sh)));
    return (uint32_t)v & ((1u << (2 * SK_M)) - 1);
}
// minimizer of a 128-bit k-mer code (the twin's m-mer p is the reverse complement of c's m-mer
// w - 1 - p: one 128-bit reversal instead of one per m-mer)
__host__ __device__ inline uint32_t minimizer_of_w(const K128 &c, int k) {
    const K128 tc = twin128(c, k);
    const int w = k - SK_M + 1;
    uint32_t v = 0xFFFFFFFFu;
    for (int p = 0; p < w; p++) {
        const uint32_t f = bits30_128(c, 2 * (k - SK_M - p)), r = bits30_128(tc, 2 * p);
        const uint32_t h = mmer_hash(f < r ? f : r);
        v = h < v ? h : v;
    }
    return min_remix_w(v);
}
__host__ __device__ inline uint64_t wide_place(const K128 &c, int k, bool mb) {
    const uint64_t h = mix128(c);
    return mb ? ((uint64_t)minimizer_of_w(c, k) << 32) | (h & 0xFFFFFFFFull) : h;
}

struct SolidIndexW {
    const SlotW *table;  // general count: the HBM table
    uint64_t capmask;
    const SubSlotW *sub;  // partitioned count (count_wide.h): bucket sub-tables of `slots` slots
    int bbits;
    unsigned int slots;
    int mb = 0;  // buckets by minimizer (count_wide.h): placement = wide_place(c, k, true)
    int k = 0;
    __device__ inline unsigned int find(const K128 &c) const {
        if (!sub) return lookup_w(table, capmask, c);
        const unsigned long long w1 = wide_w1(c), w2 = wide_w2(c);
        const uint64_t h = wide_place(c, k, mb != 0);
        const SubSlotW *r = sub + (bbits ? (h >> (64 - bbits)) : 0ull) * slots;
        unsigned int slot = (unsigned int)(((uint64_t)(uint32_t)h * slots) >> 32);  // wide_slot0
        for (unsigned int probe = 0; probe < slots; probe++) {
            const ulonglong2 ww = *reinterpret_cast<const ulonglong2 *>(&r[slot].w1);
            if (ww.x == 0) return NONE32;
            if (ww.x == w1 && ww.y == w2) return r[slot].id;
            slot = slot + 1 == slots ? 0u : slot + 1;
        }
        return NONE32;
    }
    struct Nb {};
    __device__ inline Nb nb_begin(const K128 &, const K128 &) const { return Nb{}; }
    __device__ inline unsigned int find_nb(const Nb &, const K128 &, const K128 &, const K128 &cy) const {
        return find(cy);
    }
};

// oriented node id: 2u + o (o = 1: twin of the canonical string); palindromes use o = 0 only
template <typename Ops>
__device__ inline typename Ops::K node_code(const typename Ops::K *dkey, unsigned int x, int k) {
    const typename Ops::K c = dkey[x >> 1];
    return (x & 1) ? Ops::twin(c, k) : c;
}
__device__ inline unsigned int twin_node(const uint8_t *upal, unsigned int x) {
    return upal[x >> 1] ? x : (x ^ 1u);
}

// links phase 1: out-degree (number of fw(x) in d, get_contig_forward:63) + the unique candidate
template <typename Ops, typename Index>
__global__ void __launch_bounds__(256) k_neighbors(Index idx, const typename Ops::K *dkey, unsigned int U, int k,
                                                   uint8_t *upal, uint8_t *outdeg, unsigned int *cand,
                                                   unsigned int *npal, const unsigned int *gate = nullptr) {
    using K = typename Ops::K;
    const K mask = Ops::mask(k);
    if (gate && *gate == 0) return;  // (gated: the fallback of the half-edge join, join_w.h)
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < 2ull * U; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        const K c = dkey[x >> 1];
        const K tc = Ops::twin(c, k);
        const bool pal = tc == c;
        if (x & 1) {
            if (pal) {  // the palindrome has a single dict entry: node 2u+1 does not exist
                outdeg[x] = 0;
                cand[x] = NONE32;
                continue;
            }
        } else {
            upal[x >> 1] = pal ? 1 : 0;
            if (pal && npal) atomicAdd(npal, 1u);
        }
        const K xs = (x & 1) ? tc : c, txs = (x & 1) ? c : tc;
        unsigned int n = 0, cd = NONE32;
        const typename Index::Nb nb = idx.nb_begin(xs, txs);
        for (uint32_t b = 0; b < 4; b++) {
            const K y = Ops::push(xs, b, mask);
            const K ty = Ops::twin_push(txs, b, k);
            const K cy = y < ty ? y : ty;
            const unsigned int u = idx.find_nb(nb, y, ty, cy);
            if (u != NONE32) {
                if (n == 0) cd = 2 * u + (y != cy ? 1u : 0u);
                n++;
            }
        }
        outdeg[x] = (uint8_t)n;
        cand[x] = n == 1 ? cd : NONE32;
    }
}

// links phase 2: x -> y iff |fw(x) in d| == 1, |bw(y) in d| == 1 and y != twin(x)
// (get_contig_forward:63-73; the cand == km / twin(km) stop is applied by the walk emulation)
// |bw(y) in d| == |fw(twin y) in d| == outdeg[twin y].
__device__ inline unsigned long long first_event(const unsigned long long *dfc, const unsigned long long *dft,
                                                 unsigned int x) {
    return (x & 1) ? dft[x >> 1] : dfc[x >> 1];
}

// A node's successor and first event side by side (k_succ / k_pred_rc): the walk's random step then
// touches one line instead of three (succ, dfc / dft).
struct alignas(16) NodeRec {
    unsigned int succ;
    unsigned int pad;
    unsigned long long fev;
};
// nrec != nullptr: also the ruler walk's node records (succ + first event)
__global__ void __launch_bounds__(256) k_succ(const uint8_t *upal, const uint8_t *outdeg, const unsigned int *cand,
                                              unsigned int N, unsigned int *succ, const unsigned long long *dfc,
                                              const unsigned long long *dft, NodeRec *nrec,
                                              const unsigned int *gate = nullptr) {
    if (gate && *gate == 0) return;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        unsigned int s = NONE32;
        const unsigned int y = cand[x];
        if (y != NONE32 && !((x & 1) && upal[x >> 1])) {
            const unsigned int ty = twin_node(upal, y);
            if (outdeg[ty] == 1 && y != twin_node(upal, x)) s = y;
        }
        succ[x] = s;
        if (nrec) {
            NodeRec r;
            r.succ = s;
            r.pad = 0;
            r.fev = first_event(dfc, dft, x);
            nrec[t] = r;
        }
    }
}

// partitioned links (multi-GPU): the successors of the oriented nodes of canonical ids
// [lo, hi) without the other ranks' out-degrees: the candidate's in-degree |bw(y) in d| =
// |fw(twin y) in d| is probed here (4 more probes) instead of read from a global outdeg
// array (same rule as k_neighbors + k_succ, get_contig_forward:63-73).
template <typename Ops, typename Index>
__global__ void __launch_bounds__(256) k_links_part(Index idx, const typename Ops::K *dkey, unsigned int lo,
                                                    unsigned int hi, int k, unsigned int *succ_out) {
    using K = typename Ops::K;
    const K mask = Ops::mask(k);
    const uint64_t n = 2ull * (hi - lo);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = 2 * lo + (unsigned int)t;
        const K c = dkey[x >> 1];
        const K tc = Ops::twin(c, k);
        const bool pal = tc == c;
        unsigned int s = NONE32;
        if (!((x & 1) && pal)) {
            const K xs = (x & 1) ? tc : c, txs = (x & 1) ? c : tc;
            unsigned int nfw = 0, cd = NONE32;
            const typename Index::Nb nb = idx.nb_begin(xs, txs);
            for (uint32_t b = 0; b < 4; b++) {
                const K y = Ops::push(xs, b, mask);
                const K ty = Ops::twin_push(txs, b, k);
                const K cy = y < ty ? y : ty;
                const unsigned int u = idx.find_nb(nb, y, ty, cy);
                if (u != NONE32) {
                    if (nfw == 0) cd = 2 * u + (y != cy ? 1u : 0u);
                    nfw++;
                }
            }
            const unsigned int tx = pal ? x : (x ^ 1u);
            if (nfw == 1 && cd != tx) {
                const K yc = dkey[cd >> 1];
                const K yt = Ops::twin(yc, k);
                const unsigned int tyn = yt == yc ? cd : (cd ^ 1u);  // twin node of the candidate
                const K tys = (tyn & 1) ? yt : yc, ttys = (tyn & 1) ? yc : yt;
                unsigned int nin = 0;
                const typename Index::Nb nb2 = idx.nb_begin(tys, ttys);
                for (uint32_t b = 0; b < 4; b++) {
                    const K z = Ops::push(tys, b, mask);
                    const K tz = Ops::twin_push(ttys, b, k);
                    const K cz = z < tz ? z : tz;
                    nin += idx.find_nb(nb2, z, tz, cz) != NONE32;
                }
                if (nin == 1) s = cd;
            }
        }
        succ_out[t] = s;
    }
}

// palindrome flags (and count) of every canonical node, when the links come from outside
template <typename Ops>
__global__ void __launch_bounds__(256) k_upal(const typename Ops::K *dkey, unsigned int U, int k, uint8_t *upal,
                                              unsigned int *npal) {
    unsigned int np = 0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < U; t += (uint64_t)gridDim.x * blockDim.x) {
        const typename Ops::K c = dkey[t];
        const bool pal = Ops::twin(c, k) == c;
        upal[t] = pal ? 1 : 0;
        np += pal;
    }
    for (int o = 32; o > 0; o >>= 1) np += __shfl_down(np, o);
    if ((threadIdx.x & 63) == 0 && np) atomicAdd(npal, np);
}


// ---- list ranking by a sparse ruling set ------------------------------------------------
// Rulers: every path head plus every node whose hash hits the sampling mask.  Each ruler
// walks its segment (up to the next ruler) serially, stamping (ruler, offset) on every node;
// the much shorter ruler list is then ranked by weighted Wyllie pointer jumping.  Cycles
// that drew no ruler are caught by later iterations with a denser sampling mask (the last
// one makes every still-unvisited node a ruler).
__device__ inline bool ruler_hash(unsigned int x, unsigned int smask) {
    return (mix64(0x9E3779B97F4A7C15ull ^ x) & smask) == 0;
}

// Ruler selection in two passes with one scan in between (deterministic ruler order, no
// contended counter): RULER_CHUNK nodes per block.
constexpr unsigned int RULER_CHUNK = 4096;

__device__ inline bool ruler_sel(const uint8_t *upal, const unsigned int *pred, const uint2 *rid, unsigned int x,
                                 unsigned int smask, int first) {
    if (((x & 1) && upal[x >> 1]) || rid[x].x != NONE32) return false;
    return (first && pred[x] == NONE32) || ruler_hash(x, smask);
}

// pred(x) = twin(succ(twin(x))) (the links are closed under twin-reversal), fused with the
// first ruler pass's counting (k_rulers_count with first = 1: every node's
// rid is still NONE then): block b handles the RULER_CHUNK nodes of chunk b
// nrec != nullptr: also the ruler walk's node records (when k_succ did not write them)
__global__ void __launch_bounds__(256) k_pred_rc(const uint8_t *upal, const unsigned int *succ, unsigned int N,
                                                 unsigned int smask, unsigned int *pred, unsigned int *bc,
                                                 const unsigned long long *dfc, const unsigned long long *dft,
                                                 NodeRec *nrec, unsigned long long *rbits) {
    const uint64_t c0 = (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < N ? c0 + RULER_CHUNK : N;
    unsigned int c = 0;
    // the first pass's ruler decisions, one bit per node (a wave's 64 consecutive nodes a word),
    // for k_rulers to read instead of re-deriving them from upal / pred / rid
    for (uint64_t t0 = c0; t0 < c1; t0 += blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        const bool valid = t < c1;
        const unsigned int x = (unsigned int)t;
        unsigned int p = NONE32;
        const bool skip = !valid || ((x & 1) && upal[x >> 1]);
        if (!skip) {
            const unsigned int sx = succ[twin_node(upal, x)];
            if (sx != NONE32) p = twin_node(upal, sx);
        }
        if (valid) pred[x] = p;
        const bool rul = !skip && (p == NONE32 || ruler_hash(x, smask));
        const unsigned long long m = __ballot(rul);
        if ((threadIdx.x & 63) == 0 && valid) rbits[t >> 6] = m;
        c += rul;
        if (nrec && valid) {
            NodeRec r;
            r.succ = succ[x];
            r.pad = 0;
            r.fev = first_event(dfc, dft, x);
            nrec[x] = r;
        }
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __shared__ unsigned int w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

__global__ void __launch_bounds__(256) k_rulers_count(const uint8_t *upal, const unsigned int *pred, unsigned int N,
                                                      unsigned int smask, int first, const uint2 *rid,
                                                      unsigned int *bc) {
    const uint64_t c0 = (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < N ? c0 + RULER_CHUNK : N;
    unsigned int c = 0;
    for (uint64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) c += ruler_sel(upal, pred, rid, (unsigned int)t, smask, first);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __shared__ unsigned int w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// bs = inclusive scan of bc; new rulers get ids nr + bs[b-1] + (rank in chunk)
__global__ void __launch_bounds__(256) k_rulers(const uint8_t *upal, const unsigned int *pred, unsigned int N,
                                                unsigned int smask, int first, const unsigned int *bs,
                                                const unsigned int *nr, uint2 *rid,
                                                unsigned int *rlist, const unsigned long long *rbits) {
    __shared__ unsigned int wsum[4];
    const uint64_t c0 = (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < N ? c0 + RULER_CHUNK : N;
    unsigned int base = *nr + (blockIdx.x ? bs[blockIdx.x - 1] : 0u);
    const unsigned int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t t0 = c0; t0 < c1; t0 += blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        bool sel;
        if (rbits)  // (first pass: k_pred_rc's bits; a wave-uniform word)
            sel = t < c1 && ((rbits[(t0 >> 6) + wid] >> lane) & 1ull);
        else
            sel = t < c1 && ruler_sel(upal, pred, rid, (unsigned int)t, smask, first);
        const unsigned long long m = __ballot(sel);
        if (lane == 0) wsum[wid] = (unsigned int)__popcll(m);
        __syncthreads();
        unsigned int off = base;
        for (unsigned int q = 0; q < wid; q++) off += wsum[q];
        const unsigned int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (sel) {
            const unsigned int i = off + (unsigned int)__popcll(m & ((1ull << lane) - 1));
            rlist[i] = (unsigned int)t;
            rid[t] = make_uint2(i, 0u);
        }
        base += tot;
        __syncthreads();
    }
}

__global__ void k_rulers_total(const unsigned int *bs, unsigned int nblk, unsigned int *nr) { *nr += bs[nblk - 1]; }

// ruler jump state (32 B): window = rulers i, P(i), .., P^{c-1}(i)
struct alignas(32) RJump {
    unsigned int a;    // P^c(i) or NONE
    unsigned int s;    // nodes in the segments of P(i)..P^{c-1}(i)  (= rank of i's node on a path)
    unsigned int h;    // last ruler of the window (the head ruler once a == NONE)
    unsigned int cm;   // min ruler node id in the window
    unsigned int cd;   // nodes from cm forward to i's node
    unsigned int len;  // nodes in i's own segment
    unsigned long long fm;  // min first event over the window's segments (incl. i's)
};
static_assert(sizeof(RJump) == 32, "rjump layout");


// Each ruler walks its segment up to the next ruler (a chain of dependent 16-B loads).
__global__ void __launch_bounds__(256) k_walk(const NodeRec *nrec, const unsigned int *rlist,
                                              unsigned int r0, const unsigned int *nr, unsigned int smask,
                                              uint2 *rid, unsigned int *nextR, RJump *rs,
                                              unsigned long long *nvisited) {
    const unsigned int r1 = *nr;
    unsigned long long seen = 0;
    for (uint64_t t = r0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < r1; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int i = (unsigned int)t;
        unsigned int v = rlist[i];
        const NodeRec a = nrec[v];
        unsigned long long fm = a.fev;
        unsigned int j = 0, nx = NONE32;
        unsigned int w = a.succ;
        for (;;) {
            if (w == NONE32) break;
            if (ruler_hash(w, smask)) {  // maybe the next ruler
                const unsigned int q = rid[w].x;
                if (q != NONE32) {
                    nx = q;
                    break;
                }
            }
            v = w;
            j++;
            const NodeRec b = nrec[v];
            w = b.succ;
            rid[v] = make_uint2(i, j);  // (ruler, offset) in one 8-B store
            fm = b.fev < fm ? b.fev : fm;
        }
        nextR[i] = nx;
        RJump r;
        r.a = NONE32;  // set from prevR by k_rjump_init
        r.s = 0;
        r.h = i;
        r.cm = rlist[i];
        r.cd = 0;
        r.len = j + 1;
        r.fm = fm;
        rs[i] = r;
        seen += j + 1;
    }
    for (int o = 32; o > 0; o >>= 1) seen += __shfl_down(seen, o);
    __shared__ unsigned long long bseen[4];  // one atomic per block, not per wave
    if ((threadIdx.x & 63) == 0) bseen[threadIdx.x >> 6] = seen;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long v = bseen[0] + bseen[1] + bseen[2] + bseen[3];
        if (v) atomicAdd(nvisited, v);
    }
}

__global__ void __launch_bounds__(256) k_rjump_init(const unsigned int *nextR, unsigned int nr, RJump *rs,
                                                    const unsigned int *dnr = nullptr) {
    if (dnr) nr = *dnr;  // (the ruler count on the device: no host read-back)
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int n = nextR[t];
        if (n != NONE32) rs[n].a = (unsigned int)t;  // prevR[next] = me (unique predecessor)
    }
}

// one weighted Wyllie round on the ruler list, two hops a round: after j takes y = src[j.a]'s
// span it takes z = src[y.a]'s too (both from the round's source state: z's segment starts where
// y's ended, so the spans stay contiguous) -- a pointer triples its span a round instead of
// doubling it, ~log3 instead of log2 launches (each ~5 us, launch-bound at ~10^5 rulers)
__global__ void __launch_bounds__(256) k_rjump(const RJump *src, RJump *dst, unsigned int nr, unsigned int N,
                                               const unsigned int *active_in, unsigned int *active_out,
                                               unsigned int *final_sel, unsigned int sel,
                                               const unsigned int *dnr = nullptr) {
    if (active_in && *active_in == 0) return;
    if (dnr) nr = *dnr;
    unsigned int act = 0;
    auto take = [&](RJump &j, const RJump &y) {
        const unsigned int back = j.s + y.len;  // nodes from ruler a's node forward to i's node
        if (y.cm < j.cm) {
            j.cm = y.cm;
            j.cd = back + y.cd;
        }
        // (saturated: on a cycle the spans pass N and stop; two hops of stopped spans could pass
        // 2^32 near the 2^31-node limit)
        const unsigned long long s2 = (unsigned long long)back + y.s;
        j.s = s2 < 0xFFFFFFFFull ? (unsigned int)s2 : 0xFFFFFFFFu;
        j.a = y.a;
        j.h = y.h;
        j.fm = y.fm < j.fm ? y.fm : j.fm;
    };
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        RJump j = src[t];
        if (j.a != NONE32 && j.s < N) {
            take(j, src[j.a]);
            if (j.a != NONE32 && j.s < N) take(j, src[j.a]);
            act += (j.a != NONE32 && j.s < N);
        }
        dst[t] = j;
    }
    // one flag store per block that still has live pointers (a per-wave atomic on one word
    // serialises at the memory side: ~4.5K waves cost ~50 us per round)
    if (__syncthreads_or(act != 0) && threadIdx.x == 0) *active_out = 1u;
    if (blockIdx.x == 0 && threadIdx.x == 0) *final_sel = sel;
}

// per-node path descriptor: PK = path key (head node for paths, min ruler node for cycles)
// with bit 31 = on a cycle; RK = rank (from the head / from the cycle key).  Path records
// at the key node: PL = path / cycle length, PM = min first event over it.
constexpr unsigned int CYC = 0x80000000u;

// The Wyllie rounds' result is in rs0 or rs1 as *sel says (read here: no host round trip).
__global__ void __launch_bounds__(256) k_finalize(const uint8_t *upal, const unsigned int *succ, const uint2 *rid,
                                                  const unsigned int *rlist, const RJump *rs0, const RJump *rs1,
                                                  const unsigned int *sel, const unsigned int *unconverged,
                                                  unsigned int N, unsigned int *PK,
                                                  unsigned int *RK, unsigned int *PL, unsigned long long *PM) {
    if (*unconverged) {  // the last Wyllie round still moved pointers (the host reports it):
        // in-range placeholders, so the later kernels index nothing outside their arrays
        for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
            PK[t] = (unsigned int)t;
            RK[t] = 0;
            PL[t] = 1;
            PM[t] = 0;
        }
        return;
    }
    const RJump *rs = (*sel & 1) ? rs1 : rs0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        const uint2 ro = rid[x];
        const unsigned int i = ro.x, j = ro.y;
        const RJump r = rs[i];
        if (r.a == NONE32) {  // path
            const unsigned int pk = rlist[r.h], rk = r.s + j;
            PK[x] = pk;
            RK[x] = rk;
            if (succ[x] == NONE32) {  // tail: its ruler's window spans the whole path
                PL[pk] = rk + 1;
                PM[pk] = r.fm;
            }
        } else {  // cycle
            PK[x] = r.cm | CYC;
            RK[x] = r.cd + j;
        }
    }
}

// cycle length / min: the ruler whose successor ruler is the key ruler closes the ring
__global__ void __launch_bounds__(256) k_cycle_len(const unsigned int *nextR, const unsigned int *rlist,
                                                   const RJump *rs0, const RJump *rs1, const unsigned int *sel,
                                                   const unsigned int *unconverged, unsigned int nr, unsigned int *PL,
                                                   unsigned long long *PM) {
    if (*unconverged) return;
    const RJump *rs = (*sel & 1) ? rs1 : rs0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        const RJump r = rs[t];
        if (r.a == NONE32) continue;
        const unsigned int n = nextR[t];
        if (n != NONE32 && rlist[n] == r.cm) {
            PL[r.cm] = r.cd + r.len;
            PM[r.cm] = r.fm;
        }
    }
}

// A node's path key and rank: per node (PK / RK), or -- the one-GPU tile ranking, round 6 --
// from its chain: LH[x] = the chain's super index (bit 31 set: an in-tile cycle or no node, whose
// PK / RK k_tile_chains wrote per node), LR[x] = the node's offset in the chain, PKs / RKs per
// chain.  No pass writes PK / RK for every node then (k_expand: 0.3 GB a step at the headline).
struct PathOf {
    const unsigned int *PK, *RK;
    const unsigned int *LH, *LR, *PKs, *RKs;
    __device__ inline unsigned int pk(unsigned int x) const {
        if (LH) {
            const unsigned int h = LH[x];
            if (!(h & 0x80000000u)) return PKs[h];
        }
        return PK[x];
    }
    __device__ inline void get(unsigned int x, unsigned int &pk, unsigned int &rk) const {
        if (LH) {
            const unsigned int h = LH[x];
            if (!(h & 0x80000000u)) {
                pk = PKs[h];
                rk = RKs[h] + LR[x];
                return;
            }
        }
        pk = PK[x];
        rk = RK[x];
    }
};
inline PathOf path_of(const unsigned int *PK, const unsigned int *RK) { return PathOf{PK, RK, nullptr, nullptr, nullptr, nullptr}; }

__device__ inline unsigned long long path_min(const PathOf &P, const unsigned long long *PM, unsigned int x) {
    return PM[P.pk(x) & ~CYC];
}

// start of each component (all_contigs:82-84): the oriented k-mer with the smallest first
// event over the path and its twin path (= the first dict entry not yet `done`).
__device__ inline bool is_start(const uint8_t *upal, const unsigned long long *dfc, const unsigned long long *dft,
                                const PathOf &PK, const unsigned long long *PM, unsigned int x,
                                unsigned long long &f, const uint8_t *excl = nullptr) {
    if ((x & 1) && upal[x >> 1]) return false;
    if (excl && excl[x >> 1]) return false;  // (extended.h: a component with one-way links)
    f = first_event(dfc, dft, x);
    // a <= f (x lies on its path), so f == min(a, b) iff f == a && a <= b: the twin path's
    // gather only for the one node a path holds at its minimum
    const unsigned long long a = path_min(PK, PM, x);
    if (f != a) return false;
    const unsigned long long b = path_min(PK, PM, twin_node(upal, x));
    return a <= b;
}

// Starts are compacted in two passes, RULER_CHUNK nodes per block: counts, one scan, then
// ballot ranks inside the chunk (deterministic order; an append counter serialises at
// ~88 atomics / us -- 4.6 ms for the 1.1 M contigs of reads with 0.5 % errors).
__global__ void __launch_bounds__(256) k_starts_count(const uint8_t *upal, const unsigned long long *dfc,
                                                      const unsigned long long *dft, const PathOf PK,
                                                      const unsigned long long *PM, unsigned int N, unsigned int *bc,
                                                      unsigned long long *smask, const uint8_t *excl = nullptr,
                                                      unsigned int n0 = 0) {
    // nodes [n0, N) (n0 > 0: a segment of the multi-GPU finish; smask bits relative to n0)
    const uint64_t c0 = n0 + (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < N ? c0 + RULER_CHUNK : N;
    unsigned int c = 0;
    // one bit per node (a wave's 64 consecutive nodes per word): k_starts_write reads the
    // decisions instead of repeating the path-minimum gathers
    for (uint64_t t0 = c0; t0 < c1; t0 += blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        unsigned long long f;
        const bool sel = t < c1 && is_start(upal, dfc, dft, PK, PM, (unsigned int)t, f, excl);
        const unsigned long long m = __ballot(sel);
        if ((threadIdx.x & 63) == 0 && t < c1) smask[(t - n0) >> 6] = m;
        c += sel;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __shared__ unsigned int w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// bs = inclusive scan of the chunk counts
__global__ void __launch_bounds__(256) k_starts_write(const uint8_t *upal, const unsigned long long *dfc,
                                                      const unsigned long long *dft, const PathOf PK,
                                                      const unsigned long long *PM, unsigned int N,
                                                      const unsigned int *bs, const unsigned long long *smask,
                                                      unsigned long long *skeys, unsigned int *svals,
                                                      unsigned int n0 = 0, unsigned int *nstarts = nullptr) {
    __shared__ unsigned int wsum[4];
    if (nstarts && blockIdx.x == 0 && threadIdx.x == 0) *nstarts = bs[gridDim.x - 1];  // (no copy launch)
    const uint64_t c0 = n0 + (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < N ? c0 + RULER_CHUNK : N;
    unsigned int base = blockIdx.x ? bs[blockIdx.x - 1] : 0u;
    const unsigned int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t t0 = c0; t0 < c1; t0 += blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        const unsigned long long m = t0 < c1 ? smask[(t0 - n0) >> 6 | (threadIdx.x >> 6)] : 0ull;  // (wave-uniform)
        const bool sel = t < c1 && ((m >> lane) & 1ull);
        const unsigned long long f = sel ? first_event(dfc, dft, (unsigned int)t) : 0ull;
        if (lane == 0) wsum[wid] = (unsigned int)__popcll(m);
        __syncthreads();
        unsigned int off = base;
        for (unsigned int q = 0; q < wid; q++) off += wsum[q];
        const unsigned int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (sel) {
            const unsigned int i = off + (unsigned int)__popcll(m & ((1ull << lane) - 1));
            skeys[i] = f;
            svals[i] = (unsigned int)t;
        }
        base += tot;
        __syncthreads();
    }
}

// geometry of the walk from start s (get_contig:47-56 + get_contig_forward:59-77):
//   kind 0 path, twin path disjoint   : contig = the path holding s, head..tail
//   kind 1 path equal to its twin     : p_0..p_n, s = p_j : p_0..p_{n-j-1} | p_{n-j+1}..p_n | all
//   kind 2 cycle, twin cycle disjoint : s, succ(s), ... (n nodes)
//   kind 3 cycle equal to its twin    : m = dist(s -> twin s): m == 0 -> all n from s,
//                                       else p_{m+1}..p_{n-1}, p_0..p_{m-1} (n-1 nodes)
struct Walk {
    unsigned int kind, n, j, m, lo, len;
};

__device__ inline Walk walk_of(const uint8_t *upal, const PathOf &P, const unsigned int *PL, unsigned int s) {
    Walk w;
    unsigned int pk, rk, pk2, rk2;
    P.get(s, pk, rk);
    const unsigned int ts = twin_node(upal, s);
    P.get(ts, pk2, rk2);
    const bool self = pk2 == pk;
    const unsigned int plen = PL[pk & ~CYC];
    w.j = rk;
    w.m = 0;
    w.lo = 0;
    if (!(pk & CYC)) {
        if (!self) {
            w.kind = 0;
            w.n = plen;
            w.len = plen;
        } else {
            w.kind = 1;
            const unsigned int n = plen - 1, j = rk;
            w.n = n;
            if (2 * j < n) {
                w.lo = 0;
                w.len = n - j;
            } else if (2 * j > n) {
                w.lo = n - j + 1;
                w.len = j;
            } else {
                w.lo = 0;
                w.len = n + 1;
            }
        }
    } else {
        const unsigned int n = plen;
        w.n = n;
        if (!self) {
            w.kind = 2;
            w.len = n;
        } else {
            w.kind = 3;
            w.m = (rk2 + n - rk) % n;
            w.len = w.m == 0 ? n : n - 1;
        }
    }
    return w;
}

__global__ void __launch_bounds__(256) k_contig_len(const uint8_t *upal, const PathOf P,
                                                    const unsigned int *PL, const unsigned int *sorted_nodes,
                                                    unsigned int nc, int k, unsigned int *cidxOf,
                                                    unsigned long long *clen, Walk *cwalk,
                                                    const unsigned int *xlen = nullptr, unsigned int *xcid = nullptr) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int s = sorted_nodes[i];
        if (xlen && (s & 0x80000000u)) {  // a start the extended path's emulation found (extended.h)
            const unsigned int j = s & 0x7FFFFFFFu;
            clen[i] = (unsigned long long)(k - 1) + xlen[j];
            xcid[j] = (unsigned int)i;
            continue;
        }
        cidxOf[P.pk(s) & ~CYC] = (unsigned int)i;
        const Walk w = walk_of(upal, P, PL, s);
        clen[i] = (unsigned long long)(k - 1) + w.len;
        cwalk[i] = w;  // k_emit reads the contig's geometry once instead of re-deriving it per node
    }
}

// a contig's walk geometry with its character offset: k_emit's one gather per node (the walk
// and the offset as two gathers cost ecoli10m_err's 26.8 M nodes a dependent random read each)
struct EWalk {
    Walk w;
    unsigned long long coff;
};
static_assert(sizeof(EWalk) == 32, "EWalk layout");
__global__ void __launch_bounds__(256) k_ewalk(const Walk *cwalk, const unsigned long long *coff, unsigned int nc,
                                               EWalk *ew) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        EWalk e;
        e.w = cwalk[i];
        e.coff = coff[i];
        ew[i] = e;
    }
}

// Few contigs (the headline: one): the order, walk geometry, offsets and emission records of
// all starts in one workgroup -- the radix sort, length, scan and k_ewalk launches it replaces
// were each a few microseconds of work behind ~10-30 us of host launch time.  Starts sorted by
// first event (bitonic in LDS; first events are distinct, so it equals the stable radix sort),
// contig i = k - 1 + its walk's node count characters at coff[i], coff[nc] = their total.
constexpr unsigned int SMALL_STARTS = 4096;
constexpr unsigned int SMALL_STARTS_NT = 1024;
__global__ void __launch_bounds__(SMALL_STARTS_NT) k_starts_small(
    const unsigned long long *skeys, const unsigned int *svals, unsigned int nc, const uint8_t *upal,
    const PathOf PO, const unsigned int *PL, int k, unsigned int *sorted,
    unsigned int *cidxOf, unsigned long long *coff, Walk *cwalk, EWalk *ew) {
    __shared__ unsigned long long s_k[SMALL_STARTS];
    __shared__ unsigned int s_v[SMALL_STARTS];
    __shared__ unsigned long long s_sum[SMALL_STARTS_NT];
    const unsigned int tid = threadIdx.x;
    unsigned int P = 1;
    while (P < nc) P <<= 1;
    for (unsigned int i = tid; i < P; i += SMALL_STARTS_NT) {
        s_k[i] = i < nc ? skeys[i] : ~0ull;
        s_v[i] = i < nc ? svals[i] : 0u;
    }
    __syncthreads();
    for (unsigned int size = 2; size <= P; size <<= 1)
        for (unsigned int stride = size >> 1; stride > 0; stride >>= 1) {
            for (unsigned int i = tid; i < P / 2; i += SMALL_STARTS_NT) {
                const unsigned int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = s_k[lo], b = s_k[hi];
                if ((a > b) == up) {
                    s_k[lo] = b;
                    s_k[hi] = a;
                    const unsigned int t = s_v[lo];
                    s_v[lo] = s_v[hi];
                    s_v[hi] = t;
                }
            }
            __syncthreads();
        }
    // four consecutive contigs a thread: walks, lengths, then one block scan of the sums
    unsigned long long len[4], run = 0;
    Walk w[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const unsigned int i = 4 * tid + u;
        len[u] = 0;
        if (i < nc) {
            const unsigned int s = s_v[i];
            sorted[i] = s;
            cidxOf[PO.pk(s) & ~CYC] = i;
            w[u] = walk_of(upal, PO, PL, s);
            len[u] = (unsigned long long)(k - 1) + w[u].len;
        }
        run += len[u];
    }
    s_sum[tid] = run;
    __syncthreads();
    for (unsigned int o = 1; o < SMALL_STARTS_NT; o <<= 1) {
        const unsigned long long add = tid >= o ? s_sum[tid - o] : 0ull;
        __syncthreads();
        s_sum[tid] += add;
        __syncthreads();
    }
    unsigned long long c = s_sum[tid] - run;  // exclusive
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const unsigned int i = 4 * tid + u;
        if (i < nc) {
            coff[i] = c;
            cwalk[i] = w[u];
            EWalk e;
            e.w = w[u];
            e.coff = c;
            ew[i] = e;
        }
        c += len[u];
    }
    if (tid == SMALL_STARTS_NT - 1) coff[nc] = s_sum[tid];
}

// emit: every node finds its contig through its path key, computes its walk position and
// writes its chars (contig_to_string:44-45: first node k chars, later nodes their last base).
template <typename Ops>
__global__ void __launch_bounds__(256) k_emit(const uint8_t *upal, const PathOf P,
                                              const unsigned int *PL, const typename Ops::K *dkey,
                                              const unsigned int *cidxOf, const EWalk *ew,
                                              unsigned int N, int k, char *chars,
                                              unsigned long long chars_bound, unsigned int *cfirst,
                                              unsigned int *clast, unsigned int *headOf, unsigned int *tailOf,
                                              unsigned int *bad, unsigned int n0 = 0) {
    for (uint64_t t = n0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = (unsigned int)t;
        if ((x & 1) && upal[x >> 1]) continue;
        unsigned int pk, rk;
        P.get(x, pk, rk);
        const unsigned int ci = cidxOf[pk & ~CYC];
        if (ci == NONE32) continue;  // the twin path of a disjoint pair carries the contig
        const EWalk e = ew[ci];
        const Walk &w = e.w;
        long long pos = -1;
        if (w.kind == 0) {
            pos = rk;
        } else if (w.kind == 1) {
            if (rk >= w.lo && rk < w.lo + w.len) pos = rk - w.lo;
        } else {
            const unsigned int i = (rk + w.n - w.j) % w.n;  // steps from s
            if (w.kind == 2 || w.m == 0) {
                pos = i;
            } else if (i > w.m) {
                pos = i - w.m - 1;
            } else if (i < w.m) {
                pos = w.n - 1 - w.m + i;
            }
        }
        if (pos < 0) continue;
        // the buffer holds the bound 2U + nc (k - 1) the host sized it for: a position past it
        // (never, for a consistent ranking) is reported instead of written
        if (e.coff + (unsigned long long)(k - 1) + (unsigned long long)pos >= chars_bound) {
            atomicOr(bad, 1u);
            continue;
        }
        const typename Ops::K code = node_code<Ops>(dkey, x, k);
        char *dst = chars + e.coff;
        if (pos == 0) {
            for (int i = 0; i < k; i++) dst[i] = Ops::chr(Ops::base(code, k, i));
            cfirst[ci] = x;
            headOf[x] = ci;
        } else {
            dst[k - 1 + pos] = Ops::chr(Ops::last(code));
        }
        if ((unsigned long long)pos == (unsigned long long)w.len - 1) {
            clast[ci] = x;
            tailOf[twin_node(upal, x)] = ci;
        }
    }
}

// GFA links (all_contigs:90-109): for y in fw(last kmer): heads[y] then tails[y];
// for z in fw(twin(first kmer)): heads[z] then tails[z].  Up to 8 per side.
template <typename Ops, typename Index>
__global__ void __launch_bounds__(256) k_gfa(Index idx, const typename Ops::K *dkey, const uint8_t *upal,
                                             const unsigned int *cfirst, const unsigned int *clast,
                                             const unsigned int *headOf, const unsigned int *tailOf, unsigned int nc,
                                             int k, long long *lk, unsigned int *lcnt) {
    using K = typename Ops::K;
    const K mask = Ops::mask(k);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        for (int side = 0; side < 2; side++) {
            const unsigned int src = side == 0 ? clast[i] : twin_node(upal, cfirst[i]);
            const K xs = node_code<Ops>(dkey, src, k), txs = Ops::twin(xs, k);
            unsigned int n = 0;
            long long *o = lk + (i * 2 + side) * 8;
            // (the four successors share w - 1 m-mers: one minimizer scan, as k_neighbors --
            // per-successor finds made k_gfa 1.27 ms on ecoli10m_err's 1.1 M contigs)
            const typename Index::Nb nb = idx.nb_begin(xs, txs);
            for (uint32_t b = 0; b < 4; b++) {
                const K y = Ops::push(xs, b, mask);
                const K ty = Ops::twin_push(txs, b, k);
                const K cy = y < ty ? y : ty;
                const unsigned int u = idx.find_nb(nb, y, ty, cy);
                if (u == NONE32) continue;
                const unsigned int oy = (y != cy) ? 2 * u + 1 : 2 * u;
                const unsigned int hh = headOf[oy], tt = tailOf[oy];
                if (hh != NONE32) o[n++] = 2ll * hh;
                if (tt != NONE32) o[n++] = 2ll * tt + 1;
            }
            lcnt[i * 2 + side] = n;
        }
    }
}

// GFA links to a dense array: loff = exclusive scan of the per-side counts (u64, 2nc + 1)
// (c8: the counts as bytes as well, <= 8 a side -- what travels to host memory)
__global__ void __launch_bounds__(256) k_lcnt64(const unsigned int *lcnt, unsigned int n2, unsigned long long *out,
                                                uint8_t *c8 = nullptr) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t <= n2; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int c = t < n2 ? lcnt[t] : 0u;
        out[t] = c;
        if (c8 && t < n2) c8[t] = (uint8_t)c;
    }
}
template <typename T>
__global__ void __launch_bounds__(256) k_links_compact(const long long *lk, const unsigned int *lcnt,
                                                       const unsigned long long *loff, unsigned int n2, T *out) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n2; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int c = lcnt[t];
        for (unsigned int j = 0; j < c; j++) out[loff[t] + j] = (T)lk[t * 8 + j];
    }
}

// Few contigs (k_starts_small's bound, n2 = 2 nc <= 8192 sides): the per-side link counts as
// bytes, their offsets and the compacted links in one workgroup, the total to *nlinks -- the
// count, scan and compaction launches with the host round trip between them in one launch
constexpr unsigned int SMALL_LINK_NT = 1024;
__global__ void __launch_bounds__(SMALL_LINK_NT) k_links_small(const long long *lk, const unsigned int *lcnt,
                                                              unsigned int n2, uint8_t *c8, uint32_t *out,
                                                              unsigned long long *nlinks) {
    __shared__ unsigned int s_sum[SMALL_LINK_NT];
    const unsigned int tid = threadIdx.x;
    unsigned int c[8], run = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const unsigned int i = 8 * tid + u;
        c[u] = i < n2 ? lcnt[i] : 0u;
        if (i < n2) c8[i] = (uint8_t)c[u];
        run += c[u];
    }
    s_sum[tid] = run;
    __syncthreads();
    for (unsigned int o = 1; o < SMALL_LINK_NT; o <<= 1) {
        const unsigned int add = tid >= o ? s_sum[tid - o] : 0u;
        __syncthreads();
        s_sum[tid] += add;
        __syncthreads();
    }
    unsigned int o = s_sum[tid] - run;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const unsigned long long side = 8ull * tid + u;
        for (unsigned int j = 0; j < c[u]; j++) out[o + j] = (uint32_t)lk[side * 8 + j];
        o += c[u];
    }
    if (tid == SMALL_LINK_NT - 1) *nlinks = s_sum[tid];
}

// ordered dict of build(): every valid oriented node with its first event (sort key)
__global__ void __launch_bounds__(256) k_dict_items(const uint8_t *upal, const unsigned long long *dfc,
                                                    const unsigned long long *dft, unsigned int N,
                                                    unsigned long long *keys, unsigned int *vals, unsigned int *n) {
    for (uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x; t0 < N; t0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        const unsigned int x = (unsigned int)t;
        const bool sel = t < N && !((x & 1) && upal[x >> 1]);
        const unsigned int i = wave_append(n, sel);  // order irrelevant: sorted by first event
        if (sel) {
            keys[i] = first_event(dfc, dft, x);
            vals[i] = x;
        }
    }
}

template <typename Ops>
__global__ void __launch_bounds__(256) k_dict_render(const unsigned int *nodes, unsigned int n,
                                                     const typename Ops::K *dkey, const unsigned int *dcnt, int k,
                                                     char *out, unsigned int *counts) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = nodes[i];
        const typename Ops::K c = node_code<Ops>(dkey, x, k);
        for (int p = 0; p < k; p++) out[i * k + p] = Ops::chr(Ops::base(c, k, p));
        counts[i] = dcnt[x >> 1];
    }
}

}  // namespace ec
