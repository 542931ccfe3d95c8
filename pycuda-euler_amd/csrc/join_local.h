// join_local.h -- the successor links joined inside the count's minimizer tables (round 6).
//
// join_w.h finds the links with the (k - 1)-mer half-edge join: every canonical key emits its
// two junction records (2U of them), bucket-sorted by the junction's hash over one or two LDS
// refine passes, then joined per bucket -- at config 5 (2e8 keys of 128 bits) ~9.5 GB of
// records written, refined and read back: 30 ms of a 105 ms step; 0.31 ms of the headline's 3.8.
//
// On minimizer-bucketed ids (the super-k-mer count, count_sk2.h; the wide minimizer count,
// count_wide.h) the records need not travel.  A junction J (a (k-1)-mer) holds w - 1 of the w
// m-mers of each k-mer it belongs to, so its minimizer is theirs unless their minimum sits at the
// one m-mer J lacks (~2 / (w + 1) of the records).  Every record goes to the table T(J) = the
// count's table of J's minimizer (top bits of min_remix / min_remix_w, as SolidIndex /
// SolidIndexW find a key's table); the keys of table b hold dense ids of one contiguous range
// (one workgroup reserved them), so the join workgroup of table b rebuilds its keys' records
// itself and only the records with T(J) != own table -- "foreign" -- pass through HBM:
//
//   k_jl_scan     per key: its table b and its junctions' tables (one minimizer loop) -> kof[u]
//                 = b << 2 | which of its two junctions are local; its foreign records appended
//                 (pad = T) with per-target counts
//                 and each table's id range from shuffles (k_jl_edges: the pairs across wave
//                 edges; a table met in two runs -- ids not grouped by table -- opens the gate)
//   (exclusive scan of the per-target counts) k_jl_scatter: foreign records grouped by target
//   k_jl_join     per table b: an LDS table keyed by junction collects its keys' local records
//                 and the foreign records sent to it, then writes the links as k_half_join
//                 (x -> y iff the junction has one id per side and y != twin(x))
//
// Every record of J goes to T(J), so a junction meets all of its records in one table -- the
// result is exact for any grouping; the minimizer grouping only makes the foreign share small.
// A table or the foreign buffer past its capacity, or ids not grouped by table, opens the gate
// (flag word): the caller's probe kernels then rewrite every successor (as after join_w.h).
#pragma once
#include "join_w.h"

namespace ec {

// a key's table and its suffix / prefix junctions' tables (half_recs: r1 / x1 suffix, r2 / x2
// prefix): the prefix junction holds m-mers 0 .. w - 2, the suffix junction 1 .. w - 1
__device__ inline void jl_tables(unsigned long long c, int k, int bits, unsigned int &tb, unsigned int &ts,
                                 unsigned int &tp) {
    const int w = k - SK_M + 1;
    constexpr uint32_t MM = (1u << (2 * SK_M)) - 1;
    const unsigned long long tc = twin64(c, k);
    uint32_t mp = 0xFFFFFFFFu, ms = 0xFFFFFFFFu;
    for (int p = 0; p < w; p++) {
        const uint32_t f = (uint32_t)(c >> (2 * (k - SK_M - p))) & MM, r = (uint32_t)(tc >> (2 * p)) & MM;
        const uint32_t h = mmer_hash(f < r ? f : r);
        if (p < w - 1) mp = h < mp ? h : mp;
        if (p > 0) ms = h < ms ? h : ms;
    }
    tb = sk_bucket_of(min_remix(mp < ms ? mp : ms), bits);
    ts = sk_bucket_of(min_remix(ms), bits);
    tp = sk_bucket_of(min_remix(mp), bits);
}
// 128-bit keys: the m-mers rolled out of the key two bits a step (m-mer p = w - 1 - q after q
// steps) and reverse-complemented in registers (bit reverse + pair swap) -- not two 128-bit
// extractions at variable shifts per m-mer (config 5: the scan was VALU-bound, ~900 VALU a key)
__device__ inline void jl_tables(const K128 &c, int k, int bits, unsigned int &tb, unsigned int &ts, unsigned int &tp) {
    const int w = k - SK_M + 1;
    constexpr uint32_t MM = (1u << (2 * SK_M)) - 1;
    unsigned long long lo = c.lo, hi = c.hi;
    uint32_t mp = 0xFFFFFFFFu, ms = 0xFFFFFFFFu;
    for (int q = 0; q < w; q++) {  // m-mer p = w - 1 - q: the prefix junction lacks q = 0, the suffix q = w - 1
        const uint32_t f = (uint32_t)lo & MM;
        uint32_t r = __builtin_bitreverse32(f ^ MM);                       // complement, bits reversed
        r = (((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1)) >> (32 - 2 * SK_M);  // base order reversed
        const uint32_t h = mmer_hash(f < r ? f : r);
        if (q > 0) mp = h < mp ? h : mp;
        if (q < w - 1) ms = h < ms ? h : ms;
        lo = (lo >> 2) | (hi << 62);
        hi >>= 2;
    }
    tb = bits ? min_remix_w(mp < ms ? mp : ms) >> (32 - bits) : 0u;
    ts = bits ? min_remix_w(ms) >> (32 - bits) : 0u;
    tp = bits ? min_remix_w(mp) >> (32 - bits) : 0u;
}

template <typename K> struct JLRec;
template <> struct JLRec<unsigned long long> { using R = RecJ64; };
template <> struct JLRec<K128> { using R = RecJ; };

// the join's state in one launch (four fills were four launches with host gaps between them,
// ~30 us of the headline step): flags and counters zeroed, table starts NONE, successors NONE,
// palindrome flags zeroed when odd k has none (upal non-null)
__global__ void __launch_bounds__(256) k_jl_init(unsigned int *flags, unsigned int nflags, unsigned int *rs,
                                                 unsigned int *cnt, unsigned int ntab, unsigned int *succ,
                                                 uint64_t nsucc, uint8_t *upal, uint64_t nupal) {
    const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = t0; i < nflags; i += st) flags[i] = 0;
    for (uint64_t i = t0; i < ntab; i += st) rs[i] = NONE32;
    for (uint64_t i = t0; i <= ntab; i += st) cnt[i] = 0;
    for (uint64_t i = t0; i < nsucc; i += st) succ[i] = NONE32;
    if (upal)
        for (uint64_t i = t0; i < nupal; i += st) upal[i] = 0;
}

// Foreign records are appended through JL_NCTR counters, 128 B apart, each owning a region of
// fcap / JL_NCTR records (a wave takes counter wave-id % JL_NCTR): one counter for every wave
// serialised at the memory side -- 0.83 ms at the headline's 7e4 waves, 34 ms at config 5's 3e6.
constexpr unsigned int JL_NCTR = 256, JL_CSTRIDE = 32;

// pass 1: per key, its table and local-junction bits into kof; foreign records appended (one
// reservation per wave) with their targets counted in fcnt.  Run bounds inside a wave from
// shuffles (rs / re; a table met twice opens the gate); the pairs across wave edges are left to
// k_jl_edges.  (No private arrays: the candidate records stay in named registers -- a
// runtime-indexed array put them in scratch, 0.83 ms at the headline.)
template <typename K>
__global__ void __launch_bounds__(256) k_jl_scan(const K *dkey, unsigned int U, int k, int bits, const uint8_t *upal,
                                                 unsigned int *kof, typename JLRec<K>::R *fout,
                                                 unsigned int *fcount, unsigned int fcap, unsigned int *fcnt,
                                                 unsigned int *rs, unsigned int *re, unsigned int *gate) {
    using R = typename JLRec<K>::R;
    const int j = k - 1, lane = threadIdx.x & 63;
    const K mj = kmask_j(j, (K *)nullptr);
    for (uint64_t t0 = (uint64_t)blockIdx.x * 256; t0 < U; t0 += (uint64_t)gridDim.x * 256) {
        const uint64_t u = t0 + threadIdx.x;
        const bool valid = u < U;
        R r1{}, r2{}, x1{}, x2{};
        bool e1 = false, e2 = false;
        unsigned int tb = 0xFFFFFFFFu, ts = 0, tp = 0;
        if (valid) {
            const K c = dkey[u];
            jl_tables(c, k, bits, tb, ts, tp);
            half_recs(c, (unsigned int)u, j, mj, upal, r1, r2, e1, e2, x1, x2);
            kof[u] = tb << 2 | (ts == tb ? 1u : 0u) | (tp == tb ? 2u : 0u);
        }
        // run bounds inside the wave
        const unsigned int tprev = __shfl_up(tb, 1), tnext = __shfl_down(tb, 1);
        if (valid && lane > 0 && tprev != tb) {
            if (atomicExch(&rs[tb], (unsigned int)u) != NONE32) atomicOr(gate, 1u);
        }
        if (valid && lane < 63 && (tnext != tb || u + 1 == U)) re[tb] = (unsigned int)u + 1;
        const bool c1 = valid && ts != tb, c2 = c1 && e1, c3 = valid && tp != tb, c4 = c3 && e2;
        const unsigned int nf = (unsigned int)c1 + c2 + c3 + c4;
        // wave prefix of the foreign counts, one reservation per wave
        unsigned int incl = nf;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        const unsigned int tot = __shfl(incl, 63);
        const unsigned int ctr = (unsigned int)((t0 >> 6) + (threadIdx.x >> 6)) % JL_NCTR, rsz = fcap / JL_NCTR;
        unsigned int base = 0;
        if (lane == 63 && tot) base = atomicAdd(&fcount[ctr * JL_CSTRIDE], tot);
        base = __shfl(base, 63);
        unsigned int p = base + incl - nf;
        const unsigned int p0 = ctr * rsz;
        auto put = [&](bool c, R x, unsigned int t) {
            if (!c) return;
            if (p < rsz) {
                x.pad = t;
                fout[p0 + p] = x;
                atomicAdd(&fcnt[t], 1u);
            } else {
                atomicOr(gate, 1u);
            }
            p++;
        };
        put(c1, r1, ts);
        put(c2, x1, ts);
        put(c3, r2, tp);
        put(c4, x2, tp);
    }
}

// run bounds across the wave edges of k_jl_scan (key pairs 64 i - 1, 64 i) and at 0 / U - 1
__global__ void __launch_bounds__(256) k_jl_edges(const unsigned int *kof, unsigned int U, unsigned int *rs,
                                                  unsigned int *re, unsigned int *gate) {
    const uint64_t ne = ((uint64_t)U + 63) / 64;  // edge i: keys 64 i - 1 | 64 i
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i <= ne; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t u = i * 64;  // first key of wave i
        const unsigned int a = u >= 1 && u - 1 < U ? kof[u - 1] >> 2 : 0xFFFFFFFFu;
        const unsigned int b = u < U ? kof[u] >> 2 : 0xFFFFFFFFu;
        if (u < U && a != b) {
            if (atomicExch(&rs[b], (unsigned int)u) != NONE32) atomicOr(gate, 1u);
        }
        if (u >= 1 && u - 1 < U && a != b) re[a] = (unsigned int)u;
    }
}

// foreign records grouped by target: position foff[t] + (the count's remaining share) - 1
// (region r of fin holds fcount[r * JL_CSTRIDE] records, capped at its size)
template <typename R>
__global__ void __launch_bounds__(256) k_jl_scatter(const R *fin, const unsigned int *fcount, unsigned int fcap,
                                                    const unsigned int *foff, unsigned int *fcnt, R *fout) {
    const unsigned int rsz = fcap / JL_NCTR;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (uint64_t)rsz * JL_NCTR;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned int r = (unsigned int)(i / rsz);
        if (i - (uint64_t)r * rsz >= min(fcount[r * JL_CSTRIDE], rsz)) continue;
        const R x = fin[i];
        const unsigned int pos = foff[x.pad] + atomicSub(&fcnt[x.pad], 1u) - 1u;
        fout[pos] = x;
    }
}

// LDS join tables: 64-bit junctions (16 B a slot) and 128-bit ones (24 B); probe loops
// wave-uniform as in k_half_join64 / k_half_join, every lane of the wave calling
template <int SLOTS> struct JLTab64 {
    unsigned long long key[SLOTS];
    unsigned int ids[2][SLOTS];
    __device__ inline void clear(int i) {
        key[i] = EMPTY_KEY;  // (a (k-1)-mer of <= 62 bits never equals it)
        ids[0][i] = ids[1][i] = NONE32;
    }
    __device__ inline unsigned int locate(const RecJ64 &r, bool valid, unsigned int *s_over) {
        unsigned int slot = (unsigned int)(((uint64_t)(uint32_t)mix64(r.key) * SLOTS) >> 32);
        unsigned long long cur = valid ? key[slot] : 0ull;
        bool miss = valid && cur != r.key;
#pragma unroll 1
        while (__any(miss)) {
            if (miss) {
                if (cur == EMPTY_KEY) {
                    if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {
                        s_over[0] = 1;
                        cur = r.key;
                    } else {
                        cur = atomicCAS(&key[slot], EMPTY_KEY, r.key);
                        if (cur == EMPTY_KEY) cur = r.key;
                        else atomicSub(&s_over[1], 1u);
                    }
                }
                if (cur != r.key) {
                    slot = slot + 1 == SLOTS ? 0u : slot + 1;
                    cur = key[slot];
                }
                miss = cur != r.key;
            }
        }
        return slot;
    }
};
template <int SLOTS> struct JLTabW {
    unsigned long long w1[SLOTS], w2[SLOTS];
    unsigned int ids[2][SLOTS];
    __device__ inline void clear(int i) {
        w1[i] = w2[i] = 0;
        ids[0][i] = ids[1][i] = NONE32;
    }
    __device__ inline unsigned int locate(const RecJ &r, bool valid, unsigned int *s_over) {
        const K128 o{r.lo, r.hi};
        const unsigned long long a1 = wide_w1(o), a2 = wide_w2(o);
        unsigned int slot = (unsigned int)(((uint64_t)(uint32_t)mix128(o) * SLOTS) >> 32);
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
                    if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {
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
        return slot;
    }
};
template <typename K, int SLOTS> struct JLTabOf;
template <int SLOTS> struct JLTabOf<unsigned long long, SLOTS> { using T = JLTab64<SLOTS>; };
template <int SLOTS> struct JLTabOf<K128, SLOTS> { using T = JLTabW<SLOTS>; };

// pass 2: per table b (one workgroup), its keys' local records and the foreign records sent to
// it joined in LDS; links written as k_half_join (succ filled with NONE32 before)
template <typename K, int SLOTS, int NT, bool ODD_K>
__global__ void __launch_bounds__(NT) k_jl_join(const K *dkey, const unsigned int *kof, const unsigned int *rs,
                                                const unsigned int *re, int k, const uint8_t *upal,
                                                const typename JLRec<K>::R *fsorted, const unsigned int *foff,
                                                unsigned int *succ, unsigned int *gate) {
    using R = typename JLRec<K>::R;
    constexpr unsigned int MANY = 0x80000000u;
    __shared__ typename JLTabOf<K, SLOTS>::T tab;
    __shared__ unsigned int s_over[2];
    const unsigned int b = blockIdx.x;
    const int j = k - 1;
    const K mj = kmask_j(j, (K *)nullptr);
    for (int i = threadIdx.x; i < SLOTS; i += NT) tab.clear(i);
    if (threadIdx.x == 0) s_over[0] = s_over[1] = 0;
    __syncthreads();
    auto add = [&](const R &r, bool valid) {
        const unsigned int slot = tab.locate(r, valid, s_over);
        if (valid) {
            const unsigned int side = r.tag >> 31, id = r.tag & 0x7FFFFFFFu;
            const unsigned int old = atomicCAS(&tab.ids[side][slot], NONE32, id);
            if (old != NONE32 && (old & ~MANY) != id) atomicOr(&tab.ids[side][slot], MANY);
        }
    };
    const unsigned int u0 = rs[b], u1 = u0 == NONE32 ? u0 : re[b];
    for (unsigned int o = u0; o < u1; o += NT) {  // the local records of this table's keys
        const unsigned int u = o + threadIdx.x;
        const bool valid = u < u1;
        R r1{}, r2{}, x1{}, x2{};
        bool e1 = false, e2 = false;
        unsigned int f = 0;
        if (valid) {
            half_recs(dkey[u], u, j, mj, upal, r1, r2, e1, e2, x1, x2);
            f = kof[u];
        }
        add(r1, (f & 1u) != 0);
        add(r2, (f & 2u) != 0);
        add(x1, e1 && (f & 1u));
        add(x2, e2 && (f & 2u));
    }
    const unsigned int f0 = foff[b], f1 = foff[b + 1];
    for (unsigned int o = f0; o < f1; o += NT) {  // the foreign records sent to it
        const bool valid = o + threadIdx.x < f1;
        R r{};
        if (valid) r = fsorted[o + threadIdx.x];
        add(r, valid);
    }
    __syncthreads();
    if (s_over[0]) {  // (uniform) the probe fallback rewrites every successor
        if (threadIdx.x == 0) atomicOr(gate, 1u);
        return;
    }
    for (int i = threadIdx.x; i < SLOTS; i += NT) {
        const unsigned int x = tab.ids[0][i], y = tab.ids[1][i];  // (NONE32 has bit 31 set too)
        if ((x | y) & MANY) continue;
        const unsigned int tx = ODD_K ? x ^ 1u : twin_node(upal, x), ty = ODD_K ? y ^ 1u : twin_node(upal, y);
        if (y == tx) continue;
        succ[x] = y;
        succ[ty] = tx;
    }
}

}  // namespace ec
