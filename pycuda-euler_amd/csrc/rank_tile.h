// rank_tile.h -- list ranking of the successor paths / cycles by tile contraction (round 4).
//
// The dense ids of the solid k-mers come out of the count bucket by bucket, each bucket a
// contiguous id range, and on the super-k-mer path a bucket holds whole minimizers: ~90 % of
// the links join two k-mers of one bucket, so they stay inside a tile of TN consecutive
// oriented node ids.  Ranking therefore runs in three steps:
//   1. k_tile_chains, one workgroup per tile: the tile's successors staged in LDS; the chains
//      of in-tile links are ranked there by pointer jumping (ceil(log2 TN) rounds, no HBM
//      traffic); a chain closed into a cycle inside the tile is finished on the spot (key = its
//      smallest node); every other chain becomes one weighted super node {head, length, min
//      first event, successor of its tail};
//   2. the super nodes (compacted in tile order) are ranked by the ruling set of graph.h with
//      weights: rulers walk their segments summing chain lengths (k_walk_s), the rulers by
//      weighted Wyllie (k_rjump, shared), cycles across tiles keyed by their smallest ruler;
//   3. k_expand: every node's path key and rank = its chain's + its offset in the chain.
// The outputs are graph.h's PK / RK / PL / PM, so starts, emission and GFA are unchanged.
// HBM traffic per node: its successor and first event read once in tile order, 8 bytes of
// chain position written and read back, PK / RK written; the random accesses of the ruler walk
// touch only the ~N/9 super nodes (one 16-B record each).
#pragma once

#include "graph.h"

namespace ec {

constexpr int RT_TN = 2048;        // oriented nodes per tile
constexpr int RT_NT = 512;         // threads per tile workgroup
constexpr int RT_PER = RT_TN / RT_NT;
constexpr int RT_ROUNDS = 11;      // 2^11 = RT_TN: chains and cycles of a tile are covered
constexpr unsigned int RT_FIN = 0x80000000u;  // LH flag: node of an in-tile cycle, finished
constexpr uint16_t RT_NONE = 0xFFFFu;

// super node of a chain: head node, successor of its tail (node id or NONE), length, min event
struct alignas(16) SuperRec {
    unsigned int head, succ, w, pad;
    unsigned long long fmin;
    unsigned long long pad2;
};
// the super list's walk record
struct alignas(16) SNodeRec {
    unsigned int succ;  // super index or NONE
    unsigned int w;     // chain length (nodes)
    unsigned long long fev;  // min first event over the chain
};

// The one-GPU ranking (round 6) compacts the chains in the same launch: each tile's chain count
// is published in a status word and its global base found by a decoupled look-back over the
// preceding tiles (a wave reads 64 of them at once; workgroups are dispatched in index order, so
// every tile it waits on is running or done).  The chains go straight to the super list, and
// LH holds the chain's super index instead of its head node -- no scan, no k_tile_compact, no
// head -> index map (SIDX).  Status word: epoch (30 bits: this call) | flag (2: 1 = the tile's
// own count, 2 = its inclusive prefix) | value (32).
struct TileLB {
    unsigned long long *status;  // ntiles words (cleared when allocated; the epoch tells calls apart)
    unsigned long long epoch;
    SuperRec *srec;              // the super list
    uint8_t *hasp;               // rank_supers_async's state, set up per chain
    uint2 *rid;
    unsigned long long *nchains; // the last tile writes M
    unsigned int *nr;            // ... and zeroes the ruler count and visit total
    unsigned long long *nvisited;
};
__device__ inline unsigned long long lb_word(unsigned long long epoch, unsigned int flag, unsigned int v) {
    return (epoch << 34) | ((unsigned long long)flag << 32) | v;
}
// wave 0 of the tile's workgroup: the exclusive prefix of the chain counts before tile t
__device__ inline unsigned long long tile_lookback(const TileLB &lb, unsigned int t, unsigned int cnt,
                                                   unsigned int lane) {
    unsigned long long *st = lb.status;
    if (lane == 0)
        __hip_atomic_store(&st[t], lb_word(lb.epoch, t == 0 ? 2u : 1u, cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long excl = 0;
    long long j0 = (long long)t - 1;
    while (j0 >= 0) {
        const long long j = j0 - (long long)lane;
        unsigned long long w = 0;
        unsigned int flag = 2;  // (lanes past tile 0: as if inclusive zero)
        if (j >= 0) {
            do {
                w = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                flag = (w >> 34) == lb.epoch ? (unsigned int)(w >> 32) & 3u : 0u;
            } while (flag == 0);
        } else {
            w = 0;
        }
        const unsigned int v = j >= 0 ? (unsigned int)w : 0u;
        const unsigned long long incl = __ballot(flag == 2);  // (never empty once j0 < 64)
        const unsigned int stop = incl ? (unsigned int)__ffsll((long long)incl) - 1u : 64u;  // nearest inclusive
        unsigned long long part = lane <= stop ? (unsigned long long)v : 0ull;
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        excl += part;
        if (incl) break;
        j0 -= 64;
    }
    if (lane == 0)
        __hip_atomic_store(&st[t], lb_word(lb.epoch, 2u, (unsigned int)(excl + cnt)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// block-wide OR over three rotating flag words in LDS the caller owns (their words free at the
// time; __syncthreads_or keeps a 256-B LDS buffer of its own, which put k_tile_chains just past
// the 40 KB of four workgroups a CU).  Round r sets f[r % 3]; thread 0 clears f[(r + 1) % 3]
// before the barrier: its last readers (round r - 2) have passed barrier r - 1, its next writers
// (round r + 1) start after barrier r
__device__ inline bool block_or3(bool v, unsigned int *f, unsigned int r) {
    if (threadIdx.x == 0) f[(r + 1) % 3] = 0;
    if (__ballot(v) && (threadIdx.x & 63) == 0) atomicOr(&f[r % 3], 1u);
    __syncthreads();
    return f[r % 3] != 0;
}

// nodes [n0, N): the tiles of a segment (the multi-GPU finish ranks its own segment's chains;
// a successor outside the segment is external like one outside the tile).  lb.status set: the
// chains compacted in this launch (above; LH = super index), else tile-local records in scratch
// for k_tile_compact (LH = head node).
__global__ void __launch_bounds__(RT_NT) k_tile_chains(const uint8_t *upal, const unsigned int *succ, unsigned int N,
                                                       const unsigned long long *dfc, const unsigned long long *dft,
                                                       unsigned int *LH, unsigned int *LR, unsigned long long *tcnt,
                                                       SuperRec *scratch, unsigned int *PK, unsigned int *RK,
                                                       unsigned int *PL, unsigned long long *PM, unsigned int n0 = 0,
                                                       const unsigned int *tb = nullptr, TileLB lb = TileLB{}) {
    // 40 KB of LDS, four workgroups a CU (round 6: 48.4 KB held three): distances and chain
    // lengths fit 16 bits in a 2048-node tile, the chain length is written by the chain's tail
    // (no 32-bit atomic), and the head counts / global base reuse the distances' words once the
    // pointer jumping is done
    __shared__ uint16_t s_ls[RT_TN], s_lp[RT_TN], s_p[RT_TN], s_mn[RT_TN];
    __shared__ __attribute__((aligned(16))) uint16_t s_cl[RT_TN];
    __shared__ unsigned long long s_cm[RT_TN];
    __shared__ __attribute__((aligned(16))) uint16_t s_d[RT_TN];
    static_assert(RT_PER * (RT_NT / 64) * 4 + 16 <= RT_TN * 2, "head counts fit the distance words");
    unsigned int (*s_wsum)[RT_NT / 64] = reinterpret_cast<unsigned int (*)[RT_NT / 64]>(s_d);
    unsigned long long &s_gbase = *reinterpret_cast<unsigned long long *>(s_d + RT_TN - 8);
    // block_or3's flags: chain-length words, written only after the pointer jumping
    unsigned int *s_or = reinterpret_cast<unsigned int *>(s_cl);
    unsigned int orr = 0;
    // tiles of RT_TN nodes from n0, or tb's tiles (k_tile_plan: cut at bucket starts, <= RT_TN)
    const unsigned int tile = blockIdx.x, tid = threadIdx.x;
    const unsigned int base = tb ? tb[tile] : n0 + tile * RT_TN;
    const unsigned int tend = tb ? tb[tile + 1] : (base + RT_TN < N ? base + RT_TN : N);
    // the tile's chain records at scratch[soff ..]: a tile's chains <= its nodes, so planned
    // tiles use their node offset (scratch of N records) and fixed ones tile * RT_TN
    const uint64_t soff = tb ? (uint64_t)(base - tb[0]) : (uint64_t)tile * RT_TN;
    if (tile == 0 && tid == 0) tcnt[gridDim.x] = 0;  // the scan's last element (no memset launch)
    unsigned int ext[RT_PER];
    unsigned long long fev[RT_PER];
    bool valid[RT_PER];
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        const unsigned int i = tid + q * RT_NT, x = base + i;
        valid[q] = x < tend && !((x & 1) && upal[x >> 1]);
        const unsigned int s = valid[q] ? succ[x] : NONE32;
        fev[q] = valid[q] ? first_event(dfc, dft, x) : NONE64;
        const bool in = s != NONE32 && s >= base && s < tend;
        s_ls[i] = in ? (uint16_t)(s - base) : RT_NONE;
        ext[q] = in ? NONE32 : s;
        s_lp[i] = RT_NONE;
        s_cm[i] = NONE64;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        const unsigned int i = tid + q * RT_NT;
        if (s_ls[i] != RT_NONE) s_lp[s_ls[i]] = (uint16_t)i;  // (in-degree <= 1)
    }
    __syncthreads();
    // pointer jumping towards the chain head (heads point to themselves); s_mn: the smallest
    // node passed (on a cycle, after the rounds: the cycle's smallest node)
    uint16_t p[RT_PER], mn[RT_PER];
    unsigned int d[RT_PER];
    if (tid == 0) s_or[0] = 0;  // (block_or3 round 0's flag; round r clears r + 1's)
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        const unsigned int i = tid + q * RT_NT;
        const uint16_t lp = s_lp[i];
        p[q] = lp == RT_NONE ? (uint16_t)i : lp;
        d[q] = lp == RT_NONE ? 0u : 1u;
        mn[q] = p[q] < i ? p[q] : (uint16_t)i;
        s_p[i] = p[q];
        s_d[i] = (uint16_t)d[q];
        s_mn[i] = mn[q];
    }
    __syncthreads();
    // (until every pointer reached its chain's head: ~log2 of the tile's longest chain rounds,
    // all RT_ROUNDS only in a tile holding a cycle, whose minimum needs them)
    for (int r = 0; r < RT_ROUNDS; r++) {
        bool more = false;
#pragma unroll
        for (int q = 0; q < RT_PER; q++) {
            const uint16_t a = p[q];
            d[q] += s_d[a];
            const uint16_t m2 = s_mn[a];
            mn[q] = m2 < mn[q] ? m2 : mn[q];
            p[q] = s_p[a];
            more |= s_lp[p[q]] != RT_NONE;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RT_PER; q++) {
            const unsigned int i = tid + q * RT_NT;
            s_p[i] = p[q];
            s_d[i] = (uint16_t)d[q];
            s_mn[i] = mn[q];
        }
        if (!block_or3(more, s_or, orr++)) break;
    }
    // nodes of in-tile cycles: their "head" still has a predecessor.  Rank them again from the
    // cycle's smallest node (the cycle cut in front of it)
    bool cyc[RT_PER];
    bool anyc = false;
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        cyc[q] = valid[q] && s_lp[p[q]] != RT_NONE;
        anyc |= cyc[q];
    }
    if (block_or3(anyc, s_or, orr++)) {
#pragma unroll
        for (int q = 0; q < RT_PER; q++) {
            const unsigned int i = tid + q * RT_NT;
            if (cyc[q]) {
                const bool key = i == mn[q];
                p[q] = key ? (uint16_t)i : s_lp[i];
                d[q] = key ? 0u : 1u;
            }
            s_p[i] = p[q];
            s_d[i] = (uint16_t)d[q];
        }
        __syncthreads();
        for (int r = 0; r < RT_ROUNDS; r++) {
#pragma unroll
            for (int q = 0; q < RT_PER; q++) {
                if (!cyc[q]) continue;
                const uint16_t a = p[q];
                d[q] += s_d[a];
                p[q] = s_p[a];
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < RT_PER; q++) {
                const unsigned int i = tid + q * RT_NT;
                if (!cyc[q]) continue;
                s_p[i] = p[q];
                s_d[i] = (uint16_t)d[q];
            }
            __syncthreads();
        }
    }
    // per chain / cycle at its head: length (written by the chain's tail, or by the cycle node
    // in front of its key), min first event; the successor of a chain's tail.  (The barrier: the
    // chain lengths overwrite block_or3's flags, which a slow wave may still be reading)
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        if (!valid[q]) continue;
        const unsigned int i = tid + q * RT_NT;
        const uint16_t h = p[q];
        if (cyc[q] ? s_ls[i] == h : s_ls[i] == RT_NONE) s_cl[h] = (uint16_t)(d[q] + 1);
        if (fev[q] < s_cm[h]) atomicMin(&s_cm[h], fev[q]);
    }
    // the heads in node order (q-major: node i = tid + q * NT): a wave's count per q
    const unsigned int lane = tid & 63, wid = tid >> 6;
    unsigned long long hm[RT_PER];
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        hm[q] = __ballot(valid[q] && !cyc[q] && d[q] == 0);
        if (lane == 0) s_wsum[q][wid] = (unsigned int)__popcll(hm[q]);
    }
    __syncthreads();
    unsigned int off = 0;
    for (int q = 0; q < RT_PER; q++)
        for (unsigned int w = 0; w < RT_NT / 64; w++) off += s_wsum[q][w];
    const bool direct = lb.status != nullptr;
    if (direct && wid == 0) {
        const unsigned long long g = tile_lookback(lb, tile, off, lane);
        if (lane == 0) {
            s_gbase = g;
            if (tile + 1 == gridDim.x) {
                *lb.nchains = g + off;
                *lb.nr = 0;
                *lb.nvisited = 0;
            }
        }
    }
    if (tile == 0 && tid == 0) tcnt[gridDim.x] = 0;  // (k_tile_compact's scan: its last element)
    __syncthreads();
    const unsigned long long gb = direct ? s_gbase : 0ull;
    SuperRec *out = direct ? lb.srec + gb : scratch + soff;
    unsigned int before = 0;  // heads of the earlier q
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        const unsigned int i = tid + q * RT_NT;
        unsigned int o = before;
        for (unsigned int w = 0; w < wid; w++) o += s_wsum[q][w];
        for (unsigned int w = 0; w < RT_NT / 64; w++) before += s_wsum[q][w];
        if ((hm[q] >> lane) & 1ull) {
            const unsigned int j = o + (unsigned int)__popcll(hm[q] & ((1ull << lane) - 1));
            // the chain's tail: the node at distance len - 1 from the head has no in-tile successor;
            // its successor is filled in below by the tail's thread
            SuperRec r;
            r.head = base + i;
            r.succ = NONE32;
            r.w = s_cl[i];
            r.pad = 0;
            r.fmin = s_cm[i];
            r.pad2 = 0;
            out[j] = r;
            if (direct) {
                lb.hasp[gb + j] = 0;
                lb.rid[gb + j] = make_uint2(NONE32, NONE32);
            }
            s_ls[i] = (uint16_t)j;  // (reused: head -> its index among the tile's heads)
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RT_PER; q++) {
        const unsigned int i = tid + q * RT_NT, x = base + i;
        if (!valid[q]) {
            if (x < tend) LH[x] = NONE32;
            continue;
        }
        const unsigned int h = base + p[q];
        if (cyc[q]) {  // finished here: path key = the cycle's smallest node
            LH[x] = h | RT_FIN;
            PK[x] = h | CYC;
            RK[x] = d[q];
            if (d[q] == 0) {
                PL[h] = s_cl[p[q]];
                PM[h] = s_cm[p[q]];
            }
        } else {
            const unsigned int j = s_ls[p[q]];
            LH[x] = direct ? (unsigned int)(gb + j) : h;
            // a chain's tail writes its external successor into the chain's record
            if (d[q] + 1 == s_cl[p[q]] && ext[q] != NONE32) out[j].succ = ext[q];
        }
        LR[x] = d[q];
    }
    if (tid == 0) tcnt[tile] = off;
}

// Tiles cut at bucket starts (the super-k-mer count marks each bucket's first dense id in
// bmark): a minimizer's k-mers share a bucket, so a chain leaves its tile only where its path
// changes minimizer, not where a fixed RT_TN boundary splits a bucket (~37 % of the headline's
// chains).  Tile t starts at canonical id t * RT_STEP rounded down to the nearest bucket start
// at most RT_TN / 2 - RT_STEP below it (else not rounded): tiles hold <= RT_TN oriented nodes.
// tb[t] = oriented start of tile t, tb[ntiles] = 2 U
constexpr unsigned int RT_STEP = 768;  // canonical ids per tile stride (RT_TN / 2 = 1024 at most)
// the owner merge's buckets hold ~600 solid keys (k_agg_bucket_ids: <= 1100 records), twice the
// count's: its segments are cut on a finer stride that may round down further
constexpr unsigned int RT_STEP_SEG = 512;
// (c0: the segment's first canonical id -- the multi-GPU finish plans its own segment, whose
// bucket starts its merge marked in segment-relative ids)
__global__ void __launch_bounds__(256) k_tile_plan(const unsigned int *bmark, unsigned int U, unsigned int ntiles,
                                                   unsigned int *tb, unsigned int c0 = 0, unsigned int step = RT_STEP) {
    const unsigned int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    if (t == 0 || t == ntiles) {
        tb[t] = 2 * (c0 + (t ? U : 0u));
        return;
    }
    const unsigned int c = t * step, lo = c - (RT_TN / 2 - step);  // (step >= RT_TN / 4: monotone cuts)
    unsigned int cut = c;
    for (int w = (int)(c >> 5); w >= (int)(lo >> 5); w--) {  // the highest bucket start in [lo, c]
        unsigned int m = bmark[w];
        if ((unsigned int)w == (c >> 5)) m &= (c & 31) == 31 ? ~0u : ((2u << (c & 31)) - 1);
        if (m) {
            const unsigned int pos = (unsigned int)w * 32 + 31 - (unsigned int)__clz((int)m);
            if (pos >= lo) cut = pos;
            break;
        }
    }
    tb[t] = 2 * (c0 + cut);
}

// tile heads -> the compact super list (tbase = exclusive scan of tcnt); SIDX[head] = its index.
// With hasp / rid (the one-GPU ranking): the super list's ruler state initialised on the way --
// hasp = 0, rid = NONE per super, the ruler count and visit total zeroed -- instead of four
// memset launches sized by a count the host has not read yet
__global__ void __launch_bounds__(256) k_tile_compact(const SuperRec *scratch, const unsigned long long *tcnt,
                                                      const unsigned long long *tbase, SuperRec *srec,
                                                      unsigned int *SIDX, uint8_t *hasp = nullptr,
                                                      uint2 *rid = nullptr, unsigned int *nr = nullptr,
                                                      unsigned long long *nvisited = nullptr,
                                                      unsigned long long *nchains = nullptr,
                                                      const unsigned int *tb = nullptr) {
    const unsigned int t = blockIdx.x;
    const unsigned int n = (unsigned int)tcnt[t];
    const unsigned long long b = tbase[t];
    const uint64_t soff = tb ? (uint64_t)(tb[t] - tb[0]) : (uint64_t)t * RT_TN;  // (as k_tile_chains)
    for (unsigned int j = threadIdx.x; j < n; j += blockDim.x) {
        const SuperRec r = scratch[soff + j];
        srec[b + j] = r;
        SIDX[r.head] = (unsigned int)(b + j);
        if (hasp) {
            hasp[b + j] = 0;
            rid[b + j] = make_uint2(NONE32, NONE32);
        }
    }
    if (nr && t == 0 && threadIdx.x == 0) {
        *nr = 0;
        *nvisited = 0;
    }
    if (nchains && t == 0 && threadIdx.x == 0) *nchains = tbase[gridDim.x];  // (rides on the next scalar read)
}

// the partitioned finish's ranking state: chain count M on the device, hasp = 0, rid = NONE
__global__ void __launch_bounds__(256) k_part_rank_init(unsigned long long *dM, unsigned int M, uint8_t *hasp, uint2 *rid,
                                                        unsigned int *nr, unsigned long long *nvisited) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *dM = M, *nr = 0, *nvisited = 0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < M; t += (uint64_t)gridDim.x * blockDim.x) {
        hasp[t] = 0;
        rid[t] = make_uint2(NONE32, NONE32);
    }
}

// SIDX[head] = index of a chain in a gathered super list (the multi-GPU finish)
__global__ void __launch_bounds__(256) k_super_index(const SuperRec *srec, unsigned int M, unsigned int *SIDX) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < M; t += (uint64_t)gridDim.x * blockDim.x)
        SIDX[srec[t].head] = (unsigned int)t;
}

// super successors as super indices (a tail's external successor starts its own chain), the
// walk records, and which super nodes have a predecessor (the path heads: none)
__global__ void __launch_bounds__(256) k_super_link(const SuperRec *srec, unsigned int M, const unsigned int *SIDX,
                                                    SNodeRec *nrec, uint8_t *hasp,
                                                    const unsigned long long *dM = nullptr) {
    if (dM) M = (unsigned int)*dM;  // (the count on the device: no host read-back)
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < M; t += (uint64_t)gridDim.x * blockDim.x) {
        const SuperRec r = srec[t];
        const unsigned int s = r.succ == NONE32 ? NONE32 : SIDX[r.succ];
        SNodeRec o;
        o.succ = s;
        o.w = r.w;
        o.fev = r.fmin;
        nrec[t] = o;
        if (s != NONE32) hasp[s] = 1;
    }
}

// ruler selection on the super list (graph.h k_rulers_count / k_rulers without palindromes)
__device__ inline bool sruler_sel(const uint8_t *hasp, const uint2 *rid, unsigned int i, unsigned int smask,
                                  int first) {
    if (rid[i].x != NONE32) return false;
    return (first && !hasp[i]) || ruler_hash(i, smask);
}
__global__ void __launch_bounds__(256) k_srulers_count(const uint8_t *hasp, unsigned int M, unsigned int smask,
                                                       int first, const uint2 *rid, unsigned int *bc,
                                                       const unsigned long long *dM = nullptr) {
    if (dM) M = (unsigned int)*dM;
    const uint64_t c0 = (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < M ? c0 + RULER_CHUNK : M;
    unsigned int c = 0;
    for (uint64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) c += sruler_sel(hasp, rid, (unsigned int)t, smask, first);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __shared__ unsigned int w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}
__global__ void __launch_bounds__(256) k_srulers(const uint8_t *hasp, unsigned int M, unsigned int smask, int first,
                                                 const unsigned int *bs, const unsigned int *nr, uint2 *rid,
                                                 unsigned int *rlist, const unsigned long long *dM = nullptr) {
    if (dM) M = (unsigned int)*dM;
    __shared__ unsigned int wsum[4];
    const uint64_t c0 = (uint64_t)blockIdx.x * RULER_CHUNK;
    const uint64_t c1 = c0 + RULER_CHUNK < M ? c0 + RULER_CHUNK : M;
    unsigned int base = *nr + (blockIdx.x ? bs[blockIdx.x - 1] : 0u);
    const unsigned int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t t0 = c0; t0 < c1; t0 += blockDim.x) {
        const uint64_t t = t0 + threadIdx.x;
        const bool sel = t < c1 && sruler_sel(hasp, rid, (unsigned int)t, smask, first);
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

// each ruler walks its segment of super nodes, offsets in nodes (chain lengths summed)
// (RJump::h carries the ruler's chain head NODE, not its ruler index: the Wyllie rounds copy it
// from the head ruler, and k_finalize_s reads a path's key without two dependent gathers)
__global__ void __launch_bounds__(256) k_walk_s(const SNodeRec *nrec, const unsigned int *rlist, unsigned int r0,
                                                const unsigned int *nr, unsigned int smask, uint2 *rid,
                                                unsigned int *nextR, RJump *rs, unsigned long long *nvisited,
                                                const SuperRec *srec) {
    const unsigned int r1 = *nr;
    unsigned long long seen = 0;
    for (uint64_t t = r0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < r1; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int i = (unsigned int)t;
        unsigned int v = rlist[i];
        const SNodeRec a = nrec[v];
        unsigned long long fm = a.fev;
        unsigned int j = 0, wl = a.w, cnt = 1, nx = NONE32;
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
            j += wl;
            const SNodeRec b = nrec[v];
            w = b.succ;
            wl = b.w;
            rid[v] = make_uint2(i, j);
            fm = b.fev < fm ? b.fev : fm;
            cnt++;
        }
        nextR[i] = nx;
        RJump r;
        r.a = NONE32;  // set from prevR by k_rjump_init
        r.s = 0;
        r.h = srec[rlist[i]].head;
        r.cm = rlist[i];
        r.cd = 0;
        r.len = j + wl;  // nodes of the segment
        r.fm = fm;
        rs[i] = r;
        seen += cnt;
    }
    for (int o = 32; o > 0; o >>= 1) seen += __shfl_down(seen, o);
    __shared__ unsigned long long bseen[4];
    if ((threadIdx.x & 63) == 0) bseen[threadIdx.x >> 6] = seen;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long v = bseen[0] + bseen[1] + bseen[2] + bseen[3];
        if (v) atomicAdd(nvisited, v);
    }
}

// per super node: path key (head node of the path, or the cycle's smallest ruler's head node |
// CYC) and rank of its chain's head; the path's length / min event at the key node
__global__ void __launch_bounds__(256) k_finalize_s(const SNodeRec *nrec, const SuperRec *srec, const uint2 *rid,
                                                    const unsigned int *rlist, const RJump *rs0, const RJump *rs1,
                                                    const unsigned int *sel, const unsigned int *unconverged,
                                                    unsigned int M, unsigned int *PKs, unsigned int *RKs,
                                                    unsigned int *PL, unsigned long long *PM,
                                                    const unsigned long long *dM = nullptr) {
    if (dM) M = (unsigned int)*dM;
    const bool bad = *unconverged != 0;  // (the host reports it; placeholders stay in range)
    const RJump *rs = (*sel & 1) ? rs1 : rs0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < M; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int v = (unsigned int)t;
        const uint2 ro = rid[v];
        if (bad || ro.x == NONE32) {  // (NONE: a chain no ruler reached -- the deferred check redoes the ranking)
            PKs[v] = srec[v].head;
            RKs[v] = 0;
            continue;
        }
        const RJump r = rs[ro.x];
        if (r.a == NONE32) {  // path
            const unsigned int pk = r.h, rk = r.s + ro.y;
            PKs[v] = pk;
            RKs[v] = rk;
            if (nrec[v].succ == NONE32) {  // tail chain: its ruler's window spans the path
                PL[pk] = rk + nrec[v].w;
                PM[pk] = r.fm;
            }
        } else {
            PKs[v] = srec[r.cm].head | CYC;
            RKs[v] = r.cd + ro.y;
        }
    }
}
__global__ void __launch_bounds__(256) k_cycle_len_s(const unsigned int *nextR, const unsigned int *rlist,
                                                     const SuperRec *srec, const RJump *rs0, const RJump *rs1,
                                                     const unsigned int *sel, const unsigned int *unconverged,
                                                     unsigned int nr, unsigned int *PL, unsigned long long *PM,
                                                     const unsigned int *dnr = nullptr) {
    if (*unconverged) return;
    if (dnr) nr = *dnr;
    const RJump *rs = (*sel & 1) ? rs1 : rs0;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nr; t += (uint64_t)gridDim.x * blockDim.x) {
        const RJump r = rs[t];
        if (r.a == NONE32) continue;
        const unsigned int n = nextR[t];
        if (n != NONE32 && rlist[n] == r.cm) {
            const unsigned int key = srec[r.cm].head;
            PL[key] = r.cd + r.len;
            PM[key] = r.fm;
        }
    }
}

// every node: its chain's path key and rank + its offset in the chain (SIDX null: LH holds the
// chain's super index itself)
__global__ void __launch_bounds__(256) k_expand(const unsigned int *LH, const unsigned int *LR, unsigned int N,
                                                const unsigned int *SIDX, const unsigned int *PKs,
                                                const unsigned int *RKs, unsigned int *PK, unsigned int *RK,
                                                unsigned int n0 = 0) {
    for (uint64_t t = n0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < N; t += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int h = LH[t];
        if (h == NONE32 || (h & RT_FIN)) continue;  // palindrome twin / in-tile cycle (done)
        const unsigned int si = SIDX ? SIDX[h] : h;
        PK[t] = PKs[si];
        RK[t] = RKs[si] + LR[t];
    }
}


// ---- multi-GPU partitioned finish (ec_graph_*_part): contig starts travel as records ----------
// a contig start found by the rank owning its node: its first event (the contig order), node,
// path key, walk geometry (graph.h walk_of, from the owner's PK / RK and the replicated PL)
struct alignas(16) StartRec {
    unsigned long long ev;
    unsigned int node, pk;
    Walk w;
    unsigned int clen, pad;
};
static_assert(sizeof(StartRec) == 48, "start record layout");

__global__ void __launch_bounds__(256) k_start_recs(const unsigned int *nodes, unsigned int n, const uint8_t *upal,
                                                    const unsigned long long *dfc, const unsigned long long *dft,
                                                    const PathOf P, const unsigned int *PL, int k,
                                                    StartRec *out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int x = nodes[i];
        StartRec r;
        r.ev = first_event(dfc, dft, x);
        r.node = x;
        r.pk = P.pk(x) & ~CYC;
        r.w = walk_of(upal, P, PL, x);
        r.clen = (unsigned int)(k - 1) + r.w.len;
        r.pad = 0;
        out[i] = r;
    }
}
__global__ void __launch_bounds__(256) k_start_keys(const StartRec *recs, unsigned int n, unsigned long long *keys,
                                                    unsigned int *vals) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        keys[i] = recs[i].ev;
        vals[i] = (unsigned int)i;
    }
}
// contig i = the i-th start in event order: its length, key -> index map, walk geometry
__global__ void __launch_bounds__(256) k_layout(const StartRec *recs, const unsigned int *order, unsigned int nc,
                                                unsigned long long *clen, unsigned int *cidxOf, Walk *cwalk) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        const StartRec r = recs[order[i]];
        clen[i] = r.clen;
        cidxOf[r.pk] = (unsigned int)i;
        cwalk[i] = r.w;
    }
}
// contig ends found by this rank as node + 1 (0 elsewhere: a sum over the ranks combines them)
__global__ void __launch_bounds__(256) k_ends_export(const unsigned int *cfirst, const unsigned int *clast, unsigned int nc,
                                                     unsigned int *ends) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        ends[i] = cfirst[i] == NONE32 ? 0u : cfirst[i] + 1;
        ends[nc + i] = clast[i] == NONE32 ? 0u : clast[i] + 1;
    }
}
// ... and back: first / last node per contig, heads / tails for the GFA lookups (k_emit's)
__global__ void __launch_bounds__(256) k_heads_from_ends(const unsigned int *ends, unsigned int nc, const uint8_t *upal,
                                                         unsigned int *cfirst, unsigned int *clast, unsigned int *headOf,
                                                         unsigned int *tailOf) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nc; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int f = ends[i] - 1, l = ends[nc + i] - 1;
        cfirst[i] = f;
        clast[i] = l;
        headOf[f] = (unsigned int)i;
        tailOf[twin_node(upal, l)] = (unsigned int)i;
    }
}

}  // namespace ec
