// superkmer.h -- minimizer-partitioned counting (super-k-mers) for N-free reads, 21 <= k <= 32.
//
// The window-record pipeline (count_part.h) moves one record per k-mer position through
// three HBM passes.  The minimizer of a k-mer -- the smallest hash over its w = k - m + 1
// canonical m-mers -- is also the minimizer of its twin (both hold the same canonical
// m-mers), so partitioning k-mers by minimizer still puts every occurrence of a canonical
// k-mer into one bucket.  Consecutive windows of a read mostly share their minimizer: a run
// of such windows (a super-k-mer, ~(w + 1) / 2 windows for random sequence) travels as ONE
// 32-B record carrying its bases 2-bit packed:
//
//   k_upsweep_sk    per read group : alphabet / N / staging checks, P, HyperLogLog of the
//                                    canonical k-mers, histogram of super-k-mers by minimizer
//   k_downsweep_sk  per read group : super-k-mer records to their (coarse bucket, group) run
//   k_refine        (count_part.h) : split into final buckets (minimizer bits of the record)
//   k_bucket_sk     per bucket     : records -> windows (balanced over the wave: lane l takes
//                                    window w0 + l of the wave's concatenated windows) -> the
//                                    LDS table of count_part.h -> solid filter -> dense arrays
//   SolidIndex      (graph.h)      : a key's bucket = top bits of its minimizer
//
// Sliding-window minima use the van Herk / Gil-Werman blocks: m-mer hashes are grouped in
// blocks of w; the minimum of a window = min(suffix-min of the previous block at the window's
// start, prefix-min of the current block at its end).  Per base: one hash, one LDS read and
// one LDS write; every w bases a suffix pass over the block.  All lanes of a tile start their
// reads together, so the block boundaries (and the suffix pass) are wave-uniform.
#pragma once
#include "count_part.h"

namespace ec {

constexpr int SK_M = 15;                        // minimizer length (canonical m-mers, odd: no palindromes)
constexpr int SK_MIN_K = 21;                    // super-k-mer mode for SK_MIN_K <= k <= 32
constexpr bool SK_DEFAULT = false;              // without EC_FLAG_SUPERKMER / EC_FLAG_WINDOW_RECORDS
constexpr int SK_W_MAX = 32 - SK_M + 1;         // windows per m-mer block (w) at k = 32
constexpr int SK_BASES = 86;                    // bases a record carries (172 bits)
constexpr int SK_R = 4;                         // downsweep windows per thread per round
constexpr unsigned int SK_CAP = 2 * TILE_READS; // records per round sorted in LDS (else direct stores)

struct MinCfg {
    int k, m, w;
    uint32_t mmask;  // 2m bits
    int msh;         // 2m - 2
    uint32_t nmax;   // windows per super-k-mer: n + k - 1 <= SK_BASES
};

inline MinCfg sk_cfg(int k) {
    MinCfg c;
    c.k = k;
    c.m = SK_M;
    c.w = k - SK_M + 1;
    c.mmask = (1u << (2 * SK_M)) - 1;
    c.msh = 2 * SK_M - 2;
    c.nmax = (uint32_t)(SK_BASES - k + 1);
    return c;
}

// m-mer order: a bijective 32-bit mix of the canonical code (equal hashes = equal m-mers).
// One multiply: the minimizer density it gives on random sequence (0.1119 at w = 17) matches
// a random order's 2 / (w + 1) as closely as murmur's three-multiply finaliser (0.1112), and
// the bucket bits come from min_remix.
__host__ __device__ inline uint32_t mmer_hash(uint32_t x) {
    x *= 0x9E3779B1u;
    return x ^ (x >> 15);
}

// the minimizer's identity as used downstream: the minimum hash remixed, so that its top bits
// (fine bin, coarse and final bucket) are uniform -- the minimum of w hashes itself crowds
// towards 0.  Bijective: runs still split exactly where the minimizer changes.
__host__ __device__ inline uint32_t min_remix(uint32_t x) {
    x ^= 0x5BD1E995u;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    x *= 0x297A2D39u;
    x ^= x >> 15;
    return x;
}

__host__ __device__ inline uint32_t rev2_32(uint32_t x) {
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// hash of the canonical form of forward m-mer f
__host__ __device__ inline uint32_t mmer_canon_hash(uint32_t f, const MinCfg &g) {
    const uint32_t r = rev2_32(f ^ g.mmask) >> (32 - 2 * g.m);
    return mmer_hash(f < r ? f : r);
}

// minimizer of k-mer code c (the graph phase's bucket of a key, the sharded path's owner):
// the twin's m-mer at offset p is the reverse complement of c's m-mer p, so one 64-bit
// reversal replaces a 32-bit one per m-mer (= mmer_canon_hash of every m-mer)
__host__ __device__ inline uint32_t minimizer_of(uint64_t c, const MinCfg &g) {
    const uint64_t tc = twin64(c, g.k);
    uint32_t v = 0xFFFFFFFFu;
    for (int p = 0; p < g.w; p++) {
        const uint32_t f = (uint32_t)(c >> (2 * (g.k - g.m - p))) & g.mmask;
        const uint32_t r = (uint32_t)(tc >> (2 * p)) & g.mmask;
        const uint32_t h = mmer_hash(f < r ? f : r);
        v = h < v ? h : v;
    }
    return min_remix(v);
}

// final bucket of a minimizer (bbits <= FINE_BITS)
__host__ __device__ inline unsigned int sk_bucket_of(uint32_t v, int bbits) { return bbits ? v >> (32 - bbits) : 0u; }

// ---- per-thread sliding minimizer over one read ------------------------------------------
struct SkMin {
    uint32_t *ring;  // this thread's LDS column: ring[q * TILE_READS], q < w
    uint32_t mf, mr, pm, n, i;
    __device__ inline void init(uint32_t *col, const MinCfg &g) {
        ring = col;
        mf = mr = 0;
        pm = 0xFFFFFFFFu;
        n = 0;
        i = 0;
        for (int q = 0; q < g.w; q++) ring[q * TILE_READS] = 0xFFFFFFFFu;
    }
    // push base code b; returns the minimum m-mer hash of the window ending at this base
    // (meaningful once k bases have been pushed; min_remix of it is the minimizer)
    __device__ inline uint32_t push(uint32_t b, const MinCfg &g) {
        mf = ((mf << 2) | b) & g.mmask;
        mr = (mr >> 2) | ((3u - b) << g.msh);
        n++;
        if (n < (uint32_t)g.m) return 0xFFFFFFFFu;
        const uint32_t h = mmer_hash(mf < mr ? mf : mr);
        pm = i == 0 ? h : min(pm, h);
        const uint32_t sn = i + 1 < (uint32_t)g.w ? ring[(i + 1) * TILE_READS] : 0xFFFFFFFFu;
        ring[i * TILE_READS] = h;
        const uint32_t v = min(sn, pm);
        if (i + 1 == (uint32_t)g.w) {  // block complete: hashes -> suffix minima
            uint32_t a = 0xFFFFFFFFu;
#pragma unroll
            for (int q = SK_W_MAX - 1; q >= 0; q--)
                if (q < g.w) {
                    a = min(a, ring[q * TILE_READS]);
                    ring[q * TILE_READS] = a;
                }
            i = 0;
        } else {
            i++;
        }
        return v;
    }
};

// ---- super-k-mer record ---------------------------------------------------------------------
// s1 = top 13 minimizer bits << 51 | n << 44 | bases; s2, s3 = bases.  The L = n + k - 1 bases
// of the run are the low 2L bits of s1:s2:s3, last base in the low bits of s3.  Window o of
// the run (o < n) is bits [2(L-o-k), 2(L-o)) of that 172-bit string.
struct alignas(16) SkRec {
    unsigned int read;
    unsigned int im;  // i0 (first window of the run in its read) | m (windows of the read) << 16
    unsigned long long s1, s2, s3;
};
static_assert(sizeof(SkRec) == 32, "super-k-mer record layout");
constexpr int SK_HDR_SHIFT = 64 - FINE_BITS;

__device__ inline unsigned int rec_bucket(const SkRec &r, int bbits) {
    return (unsigned int)(r.s1 >> SK_HDR_SHIFT) >> (FINE_BITS - bbits);
}
__device__ inline unsigned int sk_windows(const SkRec &r) { return (unsigned int)(r.s1 >> 44) & 0x7Fu; }

struct StoreSk {
    SkRec *p;
    __device__ inline SkRec load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const SkRec &r) const {
        uint4 *d = reinterpret_cast<uint4 *>(p + i);
        const uint4 *v = reinterpret_cast<const uint4 *>(&r);
        d[0] = v[0];
        d[1] = v[1];
    }
};

// ---- upsweep ----------------------------------------------------------------------------------
// As k_upsweep, but the histogram counts super-k-mers by minimizer.  A read with 'N' or a byte
// outside ACGTN sets lens[2]: the host then reruns the window-record upsweep (super-k-mers need
// N-free reads).  Tiles too long for the stage read global memory.
__global__ void __launch_bounds__(TILE_READS) k_upsweep_sk(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                          MinCfg mc, uint64_t gsize, unsigned int *hist,
                                                          uint8_t *hll_blocks, unsigned long long *npos,
                                                          unsigned long long *bad, unsigned int *maxlocal,
                                                          unsigned int *skew, unsigned int *lens,
                                                          unsigned long long *nrec) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_BYTES + 16];
    __shared__ unsigned int h_cnt[FINE / 2];
    __shared__ unsigned int h_reg[1 << HLL_REG_BITS];
    __shared__ uint32_t ring[SK_W_MAX * TILE_READS];
    for (int i = threadIdx.x; i < FINE / 2; i += blockDim.x) h_cnt[i] = 0;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x) h_reg[i] = 0;
    const uint64_t g = blockIdx.x;
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    const int k = mc.k;
    const uint64_t mask = kmask64(k);
    const int sh = 2 * (k - 1);
    const uint32_t km1 = (uint32_t)(k - 1);
    unsigned long long mypos = 0, myrec = 0;
    unsigned int mymax = 0, myskew = 0, mynonclean = 0;
    auto bin = [&](uint32_t v) {
        const uint32_t f = min_remix(v) >> (32 - FINE_BITS);
        const uint32_t sh16 = (f & 1) * 16;
        const uint32_t old = atomicAdd(&h_cnt[f >> 1], 1u << sh16);
        myskew |= ((old >> sh16) & 0xFFFFu) >= 0xFFFEu;
        myrec++;
    };
    for_group_reads(buf, off, g0, g1, stage,
                    [&](bool staged, const LdsRead &rv, const LdsReader &lr, uint64_t r, uint64_t s, uint64_t len) {
        uint32_t flags = 0;
        if (staged) {
            flags = read_flags(rv, (uint32_t)len);
        } else {  // tile too long for the stage: read global memory
            ByteReader br(buf);
            for (uint64_t t = 0; t < len; t++) {
                const uint32_t c = br(s + t);
                flags |= (c == 'N') | (((is_acgt(c) | (c == 'N')) ^ 1u) << 1);
            }
        }
        if (flags != 0) {
            mynonclean = 1;
            if (flags & 2) {  // report the first byte outside ACGTN
                auto scan = [&](auto &rd) {
                    for (uint64_t t = 0; t < len; t++)
                        if (base_code(rd(s + t)) == 5) {
                            atomicMin(bad, (unsigned long long)(s + t));
                            break;
                        }
                };
                if (staged) {
                    LdsReader l2 = lr;
                    scan(l2);
                } else {
                    ByteReader br(buf);
                    scan(br);
                }
            }
            return;
        }
        if (len < (uint64_t)k) return;
        const uint32_t m = (uint32_t)(len - k + 1);
        mypos += m;
        mymax = max(mymax, 2 * m - 1);
        SkMin mz;
        mz.init(ring + threadIdx.x, mc);
        uint64_t fwd = 0, rc = 0;
        uint32_t runv = 0, runn = 0;
        auto step = [&](uint32_t b, uint32_t t) {
            fwd = ((fwd << 2) | b) & mask;
            rc = (rc >> 2) | ((uint64_t)(3u - b) << sh);
            const uint32_t v = mz.push(b, mc);
            if (t < km1) return;
            const uint64_t c = fwd < rc ? fwd : rc;
            const uint64_t h = mix64(c);
            const uint32_t j = (uint32_t)(h >> (64 - HLL_REG_BITS));
            const uint32_t rho = (uint32_t)__clzll((long long)((h << HLL_REG_BITS) | (1ull << (HLL_REG_BITS - 1)))) + 1;
            if (rho > h_reg[j]) atomicMax(&h_reg[j], rho);
            if (runn && (v != runv || runn == mc.nmax)) {
                bin(runv);
                runn = 0;
            }
            if (!runn) runv = v;
            runn++;
        };
        if (staged) {
            const uint32_t full = (uint32_t)len >> 2;
            for (uint32_t i = 0; i < full; i++) {
                const uint32_t c4 = rv.chunk(i);
#pragma unroll
                for (int q = 0; q < 4; q++) step(code2(c4 >> (8 * q)), 4 * i + q);
            }
            if (len & 3) {
                const uint32_t c4 = rv.chunk(full);
                for (uint32_t q = 0; q < ((uint32_t)len & 3); q++) step(code2(c4 >> (8 * q)), 4 * full + q);
            }
        } else {
            ByteReader br(buf);
            for (uint32_t t = 0; t < (uint32_t)len; t++) step(code2(br(s + t)), t);
        }
        if (runn) bin(runv);
    });
    for (int o = 32; o > 0; o >>= 1) {
        mypos += __shfl_down(mypos, o);
        myrec += __shfl_down(myrec, o);
        mymax = max(mymax, (unsigned int)__shfl_down(mymax, o));
        myskew |= (unsigned int)__shfl_down(myskew, o);
        mynonclean |= (unsigned int)__shfl_down(mynonclean, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (mypos) atomicAdd(npos, mypos);
        if (myrec) atomicAdd(nrec, myrec);
        if (mymax) atomicMax(maxlocal, mymax);
        if (myskew) atomicOr(skew, 1u);
        if (mynonclean) atomicOr(&lens[2], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < FINE; i += blockDim.x) hist[g * FINE + i] = (h_cnt[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x)
        hll_blocks[g * (1 << HLL_REG_BITS) + i] = (uint8_t)h_reg[i];
}

// ---- downsweep: super-k-mer records to their (coarse bucket, group) runs -----------------------
// Reads advance in lock-step rounds of SK_R windows.  A run closes at most once per window
// (emitted into the register slot of that window) plus once at the read's end (slot SK_R).
// The round's records get their rank in their coarse bucket from an LDS counter; a block scan
// reserves each bucket's run; up to SK_CAP records are sorted through LDS so the stores come out
// as contiguous runs, a larger round stores directly.  The run splitting is the upsweep's.
struct SkPend {
    uint32_t v, i0, n;
    unsigned long long a1, a2, a3;
};

__global__ void __launch_bounds__(TILE_READS) k_downsweep_sk(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                            MinCfg mc, uint64_t gsize, uint64_t ngroups, int cbits,
                                                            const unsigned long long *offs, SkRec *recs,
                                                            uint64_t read_base) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_BYTES + 16];
    __shared__ uint32_t ring[SK_W_MAX * TILE_READS];
    __shared__ SkRec sorted[SK_CAP];
    __shared__ uint8_t sbk[SK_CAP];
    __shared__ unsigned int bcnt[1 << DS_MAX_CBITS], bbeg[1 << DS_MAX_CBITS];
    __shared__ unsigned long long cur[1 << DS_MAX_CBITS], gbase[1 << DS_MAX_CBITS];
    __shared__ unsigned int s_rounds, s_total, s_wave[TILE_READS / 64];
    const uint64_t g = blockIdx.x;
    const int C = 1 << cbits;
    const unsigned int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int k = mc.k;
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    for (uint64_t r0 = g0; r0 < g1; r0 += TILE_READS) {
        const uint64_t r1 = min(r0 + TILE_READS, g1);
        __syncthreads();
        for (int c = tid; c < C; c += TILE_READS) {
            if (r0 == g0) cur[c] = offs[(uint64_t)c * ngroups + g];
            bcnt[c] = 0;
        }
        if (tid == 0) s_rounds = 0;
        uint64_t base = 0;
        const bool staged = stage_tile(buf, off, r0, r1, stage, base);
        __syncthreads();
        const uint64_t r = r0 + tid;
        uint32_t m = 0;
        uint64_t s = 0;
        if (r < r1) {
            s = off[r];
            const uint64_t len = off[r + 1] - s;
            m = len >= (uint64_t)k ? (uint32_t)(len - k + 1) : 0u;
        }
        const uint32_t rel = (uint32_t)(s - base);
        ByteReader br(buf);  // unstaged tiles (long reads): global memory
        auto byte = [&](uint32_t t) -> uint32_t { return staged ? stage[rel + t] : br(s + t); };
        if (m) atomicMax(&s_rounds, (m + SK_R - 1) / SK_R);
        SkMin mz;
        mz.init(ring + tid, mc);
        unsigned long long a1 = 0, a2 = 0, a3 = 0;  // the read's latest bases, newest lowest
        auto append = [&](uint32_t b) {
            a1 = (a1 << 2) | (a2 >> 62);
            a2 = (a2 << 2) | (a3 >> 62);
            a3 = (a3 << 2) | b;
        };
        uint32_t t = 0, w = 0, runv = 0, runn = 0, runi = 0;
        if (m)
            for (; t < (uint32_t)(k - 1); t++) {
                const uint32_t b = code2(byte(t));
                mz.push(b, mc);
                append(b);
            }
        __syncthreads();
        const unsigned int nrounds = s_rounds;
        const unsigned int im_m = m << 16;
        for (unsigned int round = 0; round < nrounds; round++) {
            SkPend pd[SK_R + 1];
            unsigned int cb[SK_R + 1], rk[SK_R + 1];
            bool has[SK_R + 1];
            auto emit = [&](int slot) {
                has[slot] = true;
                const uint32_t mv = min_remix(runv);
                pd[slot] = SkPend{mv, runi, runn, a1, a2, a3};
                cb[slot] = cbits ? (mv >> (32 - cbits)) : 0u;
                rk[slot] = atomicAdd(&bcnt[cb[slot]], 1u);
            };
#pragma unroll
            for (int j = 0; j <= SK_R; j++) has[j] = false;
#pragma unroll
            for (int j = 0; j < SK_R; j++) {
                if (w < m) {
                    const uint32_t b = code2(byte(t));
                    const uint32_t v = mz.push(b, mc);
                    if (runn && (v != runv || runn == mc.nmax)) {
                        emit(j);
                        runn = 0;
                    }
                    if (!runn) {
                        runv = v;
                        runi = w;
                    }
                    runn++;
                    append(b);
                    t++;
                    w++;
                    if (w == m) emit(SK_R);
                }
            }
            __syncthreads();
            const unsigned int vv = (int)tid < C ? bcnt[tid] : 0u;
            unsigned int incl = vv;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if ((int)lane >= o) incl += u;
            }
            if (lane == 63) s_wave[wid] = incl;
            __syncthreads();
            unsigned int before = 0;
            for (unsigned int q = 0; q < wid; q++) before += s_wave[q];
            if ((int)tid < C) {
                bbeg[tid] = before + incl - vv;
                gbase[tid] = cur[tid];
                cur[tid] += vv;
            }
            if (tid == TILE_READS - 1) s_total = before + incl;
            __syncthreads();
            const unsigned int total = s_total;
            auto make = [&](const SkPend &p) {
                SkRec x;
                x.read = (unsigned int)(r + read_base);
                x.im = p.i0 | im_m;
                x.s1 = (p.a1 & ((1ull << 44) - 1)) | ((unsigned long long)p.n << 44) |
                       ((unsigned long long)(p.v >> (32 - FINE_BITS)) << SK_HDR_SHIFT);
                x.s2 = p.a2;
                x.s3 = p.a3;
                return x;
            };
            if (total <= SK_CAP) {
#pragma unroll
                for (int j = 0; j <= SK_R; j++)
                    if (has[j]) {
                        const unsigned int p = bbeg[cb[j]] + rk[j];
                        sorted[p] = make(pd[j]);
                        sbk[p] = (uint8_t)cb[j];
                    }
                __syncthreads();
                for (unsigned int i = tid; i < total; i += TILE_READS) {
                    const unsigned int c = sbk[i];
                    recs[gbase[c] + (i - bbeg[c])] = sorted[i];
                }
            } else {
#pragma unroll
                for (int j = 0; j <= SK_R; j++)
                    if (has[j]) recs[gbase[cb[j]] + rk[j]] = make(pd[j]);
            }
            if ((int)tid < C) bcnt[tid] = 0;
            __syncthreads();
        }
    }
}

// ---- bucket pass over super-k-mers -------------------------------------------------------------
// The block stages SK_CH records at a time in LDS with the exclusive scan of their window
// counts; waves then take 64-window chunks of the concatenation from an LDS counter and lane l
// handles window w0 + l -- all lanes insert whatever the run lengths.  Records are found
// without a search: staging notes the record holding each chunk's first window (chunk_first),
// lane j ORs a bit at (pre - w0) into the wave's mask for the j-th following record if it starts
// inside the chunk, and the record of window w0 + l is chunk_first + popcount(mask & bits <= l).
// The k-mer is a shift out of the record's packed bases.  Events as window.h: lf = i0 + o,
// lr = 2m - 1 - lf.  Slots within the bucket: sk_slot (cheaper than mix64; SolidIndex matches).
__device__ inline unsigned long long shr128(unsigned long long hi, unsigned long long lo, unsigned int s) {
    return s ? (lo >> s) | (hi << (64 - s)) : lo;
}

// window o of super-k-mer x (L = n + k - 1 packed bases)
__device__ inline unsigned long long sk_window(const SkRec &x, unsigned int o, int k) {
    const unsigned int L = sk_windows(x) + (unsigned int)k - 1;
    const unsigned int s = 2 * (L - o - (unsigned int)k);
    const unsigned long long v =
        s < 64 ? shr128(x.s2, x.s3, s) : (s < 128 ? shr128(x.s1, x.s2, s - 64) : x.s1 >> (s - 128));
    return v & kmask64(k);
}

// first probe slot of canonical key c in a super-k-mer bucket table (top bits used)
__host__ __device__ inline unsigned int sk_slot(unsigned long long c) {
    return (unsigned int)c * 0x9E3779B1u + (unsigned int)(c >> 32) * 0x85EBCA77u;
}

template <int SLOTS>
__global__ void __launch_bounds__(BUCKET_THREADS) k_bucket_sk(const SkRec *recs, const unsigned long long *bstart,
                                                             int k, long long limit, unsigned long long *dkey,
                                                             unsigned int *dcnt, unsigned long long *dfc,
                                                             unsigned long long *dft, SubSlot *sub,
                                                             unsigned int *nsolid, unsigned long long *ndistinct,
                                                             unsigned int *overflow) {
    constexpr unsigned int CH = SLOTS <= 2048 ? 1024 : 768;  // records staged (<= BUCKET_THREADS)
    constexpr unsigned int NCH = (CH * 127 + 63) / 64 + 1;   // 64-window chunks of CH records
    constexpr int SBITS = SLOTS == 2048 ? 11 : 12;
    constexpr unsigned int NW = BUCKET_THREADS / 64;
    __shared__ LTab<SLOTS> tab;
    __shared__ unsigned int s_over[2];
    __shared__ SkRec wrec[CH];
    __shared__ unsigned int wpre[CH + 1];
    __shared__ unsigned short chunk_first[NCH];
    __shared__ unsigned long long wmask[NW];
    __shared__ unsigned int s_next, s_wsum[NW];
    const unsigned int b = blockIdx.x;
    lds_table_init<SLOTS>(tab, s_over);
    const uint64_t r0 = bstart[b], r1 = bstart[b + 1];
    const unsigned int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t c0 = r0; c0 < r1; c0 += CH) {
        const unsigned int nrec = (unsigned int)min<uint64_t>(CH, r1 - c0);
        unsigned int n = 0;
        if (threadIdx.x < nrec) {
            const SkRec x = recs[c0 + threadIdx.x];
            wrec[threadIdx.x] = x;
            n = sk_windows(x);
        }
        // block exclusive scan of the window counts
        unsigned int incl = n;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int u = __shfl_up(incl, o);
            if ((int)lane >= o) incl += u;
        }
        if (lane == 63) s_wsum[wid] = incl;
        if (threadIdx.x == 0) s_next = 0;
        __syncthreads();
        unsigned int before = 0, T = 0;
        for (unsigned int q = 0; q < NW; q++) {
            const unsigned int v = s_wsum[q];
            before += q < wid ? v : 0u;
            T += v;
        }
        const unsigned int pre = before + incl - n;
        if (threadIdx.x < nrec) {
            wpre[threadIdx.x] = pre;
            for (unsigned int c = (pre + 63) >> 6; c << 6 < pre + n; c++) chunk_first[c] = (unsigned short)threadIdx.x;
        }
        if (threadIdx.x == 0) wpre[nrec] = T;
        __syncthreads();
        const unsigned int nchunks = (T + 63) >> 6;
        for (;;) {
            unsigned int ch = 0;
            if (lane == 0) ch = atomicAdd(&s_next, 1u);
            ch = __builtin_amdgcn_readfirstlane(ch);
            if (ch >= nchunks) break;
            const unsigned int w0 = ch << 6;
            const unsigned int r = chunk_first[ch];
            if (lane == 0) wmask[wid] = 0;
            const unsigned int j = r + 1 + lane;
            if (j < nrec) {
                const unsigned int p = wpre[j];
                if (p < w0 + 64) atomicOr(&wmask[wid], 1ull << (p - w0));
            }
            const unsigned long long mask = wmask[wid];
            const unsigned int w = w0 + lane;
            if (w < T) {
                const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
                const unsigned int o = r + (unsigned int)__popcll(mask & upto);
                const SkRec x = wrec[o];
                const unsigned int off = w - wpre[o];
                const unsigned long long fwd = sk_window(x, off, k);
                const unsigned long long rc = twin64(fwd, k);
                const unsigned int i0 = x.im & 0xFFFFu, m = x.im >> 16;
                const unsigned int lf = i0 + off, lr = 2 * m - 1 - lf;
                const unsigned long long rd = (unsigned long long)x.read << 32;
                const bool f = fwd < rc;
                const unsigned long long c = f ? fwd : rc;
                const unsigned int add = fwd == rc ? 2u : 1u;  // even-k palindrome: inserted twice,
                const unsigned int lC = f || fwd == rc ? lf : lr, lT = f && fwd != rc ? lr : lf;  // at lf
                lds_insert<SLOTS>(tab, s_over, c, sk_slot(c) >> (32 - SBITS), add, rd | lC, rd | lT);
            }
        }
        __syncthreads();
    }
    lds_table_finish<SLOTS>(tab, s_over, b, limit, dkey, dcnt, dfc, dft, sub, nsolid, ndistinct, overflow);
}

}  // namespace ec
