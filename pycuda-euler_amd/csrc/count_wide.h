// count_wide.h -- partitioned (LDS-table) counting for 128-bit keys, 32 < k <= 63 (BASELINE
// config 5: k = 51, 150 bp reads).  The same four passes as count_part.h -- upsweep (fine
// histogram by hash + HyperLogLog), downsweep (records to their (coarse bucket, group) runs,
// LDS counting sort per batch), refine (coarse -> final buckets, k_refine<RecW>), bucket
// (one LDS table per final bucket) -- on 24-B records {key lo, key hi, read, lC | lT << 16}.
// The bucket hash is mix128 of the canonical key throughout.  Taken for N-free reads whose
// 256-read tiles fit the 40 KB stage (reads up to ~160 bp); other inputs keep the HBM-table
// path of wide.h.
#pragma once
#include <type_traits>
#include "count_part.h"
#include "graph.h"
#include "superkmer.h"
#include "wide.h"

namespace ec {

// ---- minimizer buckets for 128-bit keys (round 4) ------------------------------------------
// With the bucket of a key = its minimizer (the smallest hash over its w = k - 14 canonical
// 15-mers, superkmer.h) instead of mix128, a bucket holds whole minimizers, so the dense ids a
// bucket gets are the k-mers of ~(w + 1) / 2-window runs of the genome: consecutive nodes of a
// path mostly share a tile of ids (rank_tile.h ranks them in LDS) -- on hash buckets every link
// leaves its tile.  The placement hash keeps mix128's low 32 bits for the slot inside a table:
//   wide_place(c) = min_remix_w(minimizer) << 32 | low 32 bits of mix128(c).
// Records carry the top 24 placement bits in the unused top bits of the key's high word (2k <=
// 104: k <= 52), so the refine levels need not recompute the minimizer (graph.h wide_place).
constexpr int WMB_MAX_K = 52;
constexpr int WMB_SHIFT = 40;  // record hi: key bits below, placement bits 32..55 above

// Per-window minimizers of reads of one length L (lane = read): window w of read r at
// wbv_at(r, w) = (r / 256) 256 M + w 256 + r % 256 (M = L - k + 1 windows): the layout the
// upsweep / downsweep read it in (lane = read of a 256-read tile, one window at a time), so
// their loads and these stores are contiguous across the lanes.  Van Herk / Gil-Werman with the
// block length W = k - 14 a template parameter, as k_skpart_w: a round is one block of W
// m-mers, their hashes and the previous block's suffix minima in registers (window rW + j =
// min(suffix_r[j], prefix_{r+1}[j - 1])).  One wave per 64 reads, staged in LDS by 16-byte
// loads.  A read of another length raises *bad (the call takes mix128 buckets).
// (First versions: every hash of a read in LDS, 35 KB a wave -- 20 ms at config 5; then
// per-lane byte loads through a register window -- 9.5 ms, divergent dependent loads.)
constexpr uint32_t WMB_MAXL = 160;
__host__ __device__ inline uint64_t wbv_at(uint64_t r, uint32_t w, uint32_t M) {
    return (r >> 8) * 256ull * M + (uint64_t)w * 256u + (r & 255u);
}
template <int W>
__global__ void __launch_bounds__(64) k_wbv(const uint8_t *buf, const uint64_t *off, uint64_t nreads, uint32_t L,
                                            uint32_t *wbv, unsigned int *bad, uint32_t *pk = nullptr, uint32_t pkd = 0) {
    __shared__ __attribute__((aligned(16))) uint8_t st[64 * WMB_MAXL + 32];
    constexpr int K = W + SK_M - 1;
    const uint32_t lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64, r1 = r0 + 64 < nreads ? r0 + 64 : nreads;
    const uint64_t b0 = off[r0], b1 = off[r1];
    const uint64_t a0 = ((uint64_t)(buf + b0)) & ~15ull, a1 = (((uint64_t)(buf + b1)) + 15) & ~15ull;
    const uint32_t n16 = (uint32_t)((a1 - a0) >> 4);
    if (n16 * 16 > sizeof st) {  // (reads of length L > WMB_MAXL are not sent here)
        if (lane == 0) *bad = 1u;
        return;
    }
    for (uint32_t i = lane; i < n16; i += 64)
        reinterpret_cast<uint4 *>(st)[i] = reinterpret_cast<const uint4 *>(a0)[i];
    __syncthreads();
    const uint64_t r = r0 + lane;
    if (r >= r1) return;
    const uint64_t s = off[r];
    if (off[r + 1] - s != L) {
        *bad = 1u;
        return;
    }
    const uint8_t *rd = st + ((uint64_t)(buf + s) - a0);
    const uint32_t M = L - K + 1, nh = L - SK_M + 1;
    constexpr uint32_t MM = (1u << (2 * SK_M)) - 1;
    uint32_t mf = 0, mr = 0, nonacgt = 0;
    uint32_t pacc = 0, pcnt = 0;  // (pk: the read's 2-bit codes, base t at bits 2 (t % 16) of dword t / 16)
    uint32_t *pout = pk ? pk + r * (uint64_t)pkd : nullptr;
    auto push = [&](uint32_t b) {
        mf = ((mf << 2) | b) & MM;
        mr = (mr >> 2) | ((3u - b) << (2 * SK_M - 2));
    };
    // (every byte of the read passes here once: a byte other than A/C/G/T flags the call as the
    // length check does -- k_upsweep_runs no longer stages the reads to look)
    auto base = [&](uint32_t c) {
        nonacgt |= is_acgt(c) ^ 1u;
        const uint32_t b = code2(c);
        if (pout) {
            pacc |= b << (2 * (pcnt & 15));
            if ((pcnt & 15) == 15) pout[pcnt >> 4] = pacc, pacc = 0;
            pcnt++;
        }
        return b;
    };
    for (uint32_t t = 0; t < SK_M - 1; t++) push(base(rd[t]));
    uint32_t S[W];
#pragma unroll
    for (int j = 0; j < W; j++) {  // block 0: m-mers 0 .. W - 1 (all exist: L >= K)
        push(base(rd[SK_M - 1 + j]));
        S[j] = mmer_hash(mf < mr ? mf : mr);
    }
#pragma unroll
    for (int j = W - 2; j >= 0; j--) S[j] = min(S[j], S[j + 1]);
    uint32_t *outp = wbv + wbv_at(r, 0, M);
    for (uint32_t w0 = 0; w0 < M; w0 += W) {
        uint32_t H[W];
        uint32_t P = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < W; j++) {
            const uint32_t w = w0 + j;
            if (w < M) outp[(uint64_t)w * 256u] = min_remix_w(min(S[j], P));
            const uint32_t e = w0 + W + j;  // m-mer of the next block
            H[j] = 0xFFFFFFFFu;
            if (e < nh) {
                push(base(rd[e + SK_M - 1]));
                H[j] = mmer_hash(mf < mr ? mf : mr);
            }
            P = min(P, H[j]);
        }
#pragma unroll
        for (int j = 0; j < W; j++) S[j] = H[j];
#pragma unroll
        for (int j = W - 2; j >= 0; j--) S[j] = min(S[j], S[j + 1]);
    }
    if (pout && (pcnt & 15)) pout[pcnt >> 4] = pacc;
    if (nonacgt) *bad = 1u;
}

constexpr int STAGE_W = 40896;  // LDS stage of the wide kernels (256 reads of <= 159 bases; upsweep in 80 KB)
constexpr int FINE_W_BITS = 14;  // fine histogram bins (16384 buckets: up to ~30 M distinct keys)
constexpr int SLOTS_W = 3328;    // LDS table slots per bucket (156 KB of 48-B slots: load <= ~0.4)
constexpr int FINE_W = 1 << FINE_W_BITS;
constexpr int DS_RW = 4;        // downsweep windows per lane per round (24-B records: 24 KB batch)
constexpr int DS_BATCH_W = TILE_READS * DS_RW;

struct alignas(8) RecW {
    unsigned long long lo, hi;
    unsigned int read;
    unsigned int ev;  // lC | lT << 16
};
static_assert(sizeof(RecW) == 24, "wide record layout");
__device__ inline K128 rkey(const RecW &r) { return K128{r.lo, r.hi}; }
__device__ inline unsigned int rec_bucket(const RecW &r, int bbits) {
    return (unsigned int)(mix128(rkey(r)) >> 32) >> (32 - bbits);
}
// minimizer-bucketed records (k <= WMB_MAX_K): placement bits 32..55 in hi's top 24 bits
struct alignas(8) RecWM : RecW {};
static_assert(sizeof(RecWM) == 24, "wide record layout");
__device__ inline K128 rkey(const RecWM &r) { return K128{r.lo, r.hi & ((1ull << WMB_SHIFT) - 1)}; }
__device__ inline unsigned int rec_bucket(const RecWM &r, int bbits) {
    return bbits ? ((unsigned int)(r.hi >> WMB_SHIFT) << 8) >> (32 - bbits) : 0u;
}
struct StoreWM {
    RecWM *p;
    __device__ inline RecWM load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const RecWM &r) const { p[i] = r; }
};
struct StoreW {
    RecW *p;
    __device__ inline RecW load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const RecW &r) const { p[i] = r; }
};

// ---- minimizer runs (round 5): one 16-B record per run of windows sharing a minimizer -------
// On minimizer buckets all windows of a read's run of one minimizer go to the same bucket, so
// the partition passes can carry the RUN {read, first window, windows, placement bits} instead
// of its windows' 24-B records: config 5's 1.25e9 windows are ~6.6e7 runs (~19 windows each),
// so the downsweep writes and the refine / third level move ~1 GB instead of 30 GB.  The bucket
// pass gathers a run's bases from the reads (still in HBM) and rolls its windows out itself.
struct alignas(16) RunWM {
    unsigned int read;   // read index of the call (0-based; + read_base in the events)
    unsigned int wn;     // first window | windows << 16
    unsigned int place;  // placement bits 32..55 (the minimizer's top 24 bits, as RecWM)
    unsigned int pad;
};
static_assert(sizeof(RunWM) == 16, "run record layout");
__device__ inline unsigned int rec_bucket(const RunWM &r, int bbits) {
    return bbits ? (r.place << 8) >> (32 - bbits) : 0u;
}
struct StoreRM {
    RunWM *p;
    __device__ inline RunWM load(uint64_t i) const { return p[i]; }
    __device__ inline void store(uint64_t i, const RunWM &r) const { p[i] = r; }
};
constexpr uint32_t RUN_MAXW = 255;  // windows a run record holds at most

__device__ inline bool stage_tile_w(const uint8_t *buf, const uint64_t *off, uint64_t r0, uint64_t r1, uint8_t *stage,
                                    uint64_t &base) {
    const uint64_t b0 = off[r0], b1 = off[r1];
    const uint64_t a0 = ((uint64_t)(buf + b0)) & ~15ull;
    const uint64_t a1 = (((uint64_t)(buf + b1)) + 15) & ~15ull;
    if (a1 - a0 > (uint64_t)STAGE_W) return false;
    base = a0 - (uint64_t)buf;
    const uint4 *src = reinterpret_cast<const uint4 *>(a0);
    uint4 *dst = reinterpret_cast<uint4 *>(stage);
    const unsigned n16 = (unsigned)((a1 - a0) >> 4);
    for (unsigned i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
    return true;
}

// one 2-bit base into the forward / reverse-complement 128-bit codes (sh = 2(k-1) >= 64)
__device__ inline void roll_w(K128 &fwd, K128 &rc, uint32_t b, const K128 &mask, int sh) {
    fwd = push128(fwd, b, mask);
    rc.lo = (rc.lo >> 2) | (rc.hi << 62);
    rc.hi = (rc.hi >> 2) | ((unsigned long long)(3u - b) << (sh - 64));
}

// ---- upsweep: fine histogram (16384 bins by mix128) + HyperLogLog, per read group ----------
// lens[2] is set when a read has an 'N' / another byte, or a tile does not fit the stage:
// the host then counts on the HBM table instead.
// RUNS (minimizer runs, MB only): the histogram counts run records -- a window opens one
// where its minimizer differs from the previous window's, or the open run holds RUN_MAXW
template <bool MB, bool RUNS = false>
__global__ void __launch_bounds__(TILE_READS) k_upsweep_w(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                          int k, uint64_t gsize, unsigned int *hist,
                                                          uint8_t *hll_blocks, unsigned long long *npos,
                                                          unsigned int *maxlocal, unsigned int *skew,
                                                          unsigned int *lens, const uint32_t *wbv, uint32_t mbM,
                                                          uint32_t smask = 0) {
    // smask (minimizer buckets): the HyperLogLog sees only the k-mers whose minimizer's low bits
    // (pv bits 12.., uniform) & smask are zero -- the estimate x (smask + 1), as the super-k-mer
    // count samples it; the canonical form and mix128 of the other windows are not computed
    // (config 5: the upsweep was compute-bound on them, 8 ms)
    static_assert(MB || !RUNS, "runs need minimizer buckets");
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_W + 16];
    __shared__ unsigned int h_cnt[FINE_W / 2];
    __shared__ unsigned int h_reg[1 << HLL_REG_BITS];
    for (int i = threadIdx.x; i < FINE_W / 2; i += blockDim.x) h_cnt[i] = 0;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x) h_reg[i] = 0;
    const uint64_t g = blockIdx.x;
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    const K128 mask = kmask128(k);
    const int sh = 2 * (k - 1);
    unsigned long long mypos = 0, myrec = 0;
    unsigned int mymax = 0, mynonclean = 0;
    for (uint64_t r0 = g0; r0 < g1; r0 += TILE_READS) {
        const uint64_t r1 = min(r0 + TILE_READS, g1);
        uint64_t base = 0;
        __syncthreads();
        const bool staged = stage_tile_w(buf, off, r0, r1, stage, base);
        __syncthreads();
        const uint64_t r = r0 + threadIdx.x;
        if (!staged) {
            mynonclean = 1;
            continue;
        }
        if (r >= r1) continue;
        const uint64_t s = off[r], len = off[r + 1] - s;
        const uint32_t rel = (uint32_t)(s - base);
        const LdsRead rv{reinterpret_cast<const uint32_t *>(stage), rel >> 2, rel & 3};
        if (read_flags(rv, (uint32_t)len) != 0) {
            mynonclean = 1;
            continue;
        }
        if (len < (uint64_t)k) continue;
        const uint32_t m = (uint32_t)(len - k + 1);
        mypos += m;
        mymax = max(mymax, 2 * m - 1);
        K128 fwd{0, 0}, rc{0, 0};
        uint32_t c4 = 0;
        uint32_t runv = 0, runl = 0;  // RUNS: the open run's minimizer and windows
        for (uint32_t t = 0; t < (uint32_t)len; t++) {
            if ((t & 3) == 0) c4 = rv.chunk(t >> 2);
            roll_w(fwd, rc, code2(c4 >> (8 * (t & 3))), mask, sh);
            if (t + 1 < (uint32_t)k) continue;
            const uint32_t pv0 = MB ? wbv[wbv_at(r, t + 1 - (uint32_t)k, mbM)] : 0u;
            const bool samp = !MB || ((pv0 >> 12) & smask) == 0;
            uint32_t hh = 0;
            if (samp) {
                const K128 c = fwd < rc ? fwd : rc;
                hh = (uint32_t)(mix128(c) >> 32);  // as k_upsweep
            }
            const uint32_t pv = MB ? pv0 : hh;
            const uint32_t f = pv >> (32 - FINE_W_BITS);
            bool open = true;
            if (RUNS) {
                open = t + 1 == (uint32_t)k || pv != runv || runl == RUN_MAXW;
                runl = open ? 1u : runl + 1;
                runv = pv;
                myrec += open;
            }
            if (open) atomicAdd(&h_cnt[f >> 1], 1u << ((f & 1) * 16));  // overflow: checked after the group
            if (samp) {
                const uint32_t j = hh >> (32 - HLL_REG_BITS);
                const uint32_t rho = (uint32_t)__clz((int)((hh << HLL_REG_BITS) | (1u << (HLL_REG_BITS - 1)))) + 1;
                if (rho > h_reg[j]) atomicMax(&h_reg[j], rho);
            }
        }
    }
    unsigned long long binsum = 0;  // bin-sum overflow check of k_upsweep
    __syncthreads();
    for (int i = threadIdx.x; i < FINE_W / 2; i += blockDim.x) binsum += (h_cnt[i] & 0xFFFFu) + (h_cnt[i] >> 16);
    if (!RUNS) myrec = mypos;
    for (int o = 32; o > 0; o >>= 1) {
        mypos += __shfl_down(mypos, o);
        myrec += __shfl_down(myrec, o);
        binsum += __shfl_down(binsum, o);
        mymax = max(mymax, (unsigned int)__shfl_down(mymax, o));
        mynonclean |= (unsigned int)__shfl_down(mynonclean, o);
    }
    __shared__ unsigned long long s_diff;
    if (threadIdx.x == 0) s_diff = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_diff, myrec - binsum);
        if (mypos) atomicAdd(npos, mypos);
        if (mymax) atomicMax(maxlocal, mymax);
        if (mynonclean) atomicOr(&lens[2], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_diff != 0) atomicOr(skew, 1u);
    for (int i = threadIdx.x; i < FINE_W; i += blockDim.x) hist[g * FINE_W + i] = (h_cnt[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x)
        hll_blocks[g * (1 << HLL_REG_BITS) + i] = (uint8_t)h_reg[i];
}

// ---- upsweep of minimizer runs without the reads (round 6) ------------------------------------
// RUNS only needs each window's minimizer (k_wbv wrote it) to find where runs open, so the reads
// are not staged and no window's k-mer is rolled: a thread a read walks its windows' wbv words
// (lane-contiguous loads) and counts run opens into the fine histogram; only the HyperLogLog's
// windows (minimizer low bits & smask == 0, see k_upsweep_w) build their canonical k-mer from the
// read bytes.  k_wbv checked every byte (A/C/G/T) and length.  The staged kernel held 80 KB of
// LDS (the 40-KB stage + histogram + registers: two workgroups a CU) and rolled every base:
// config 5's upsweep 7.8 ms.
__global__ void __launch_bounds__(TILE_READS) k_upsweep_runs(const uint8_t *buf, const uint64_t *off,
                                                             uint64_t nreads, int k, uint64_t gsize, unsigned int *hist,
                                                             uint8_t *hll_blocks, unsigned long long *npos,
                                                             unsigned int *maxlocal, unsigned int *skew,
                                                             const uint32_t *wbv, uint32_t mbM, uint32_t smask) {
    __shared__ unsigned int h_cnt[FINE_W / 2];
    __shared__ unsigned int h_reg[1 << HLL_REG_BITS];
    for (int i = threadIdx.x; i < FINE_W / 2; i += blockDim.x) h_cnt[i] = 0;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x) h_reg[i] = 0;
    __syncthreads();
    const uint64_t g = blockIdx.x;
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    const K128 mask = kmask128(k);
    const int sh = 2 * (k - 1);
    unsigned long long mypos = 0, myrec = 0;
    unsigned int mymax = 0;
    for (uint64_t r = g0 + threadIdx.x; r < g1; r += TILE_READS) {
        const uint64_t s = off[r];
        const uint64_t len = off[r + 1] - s;
        if (len < (uint64_t)k) continue;
        const uint32_t m = (uint32_t)(len - k + 1);
        mypos += m;
        mymax = max(mymax, 2 * m - 1);
        uint32_t runv = 0, runl = 0;
        K128 fwd{0, 0}, rc{0, 0};
        bool have = false;  // fwd / rc hold the previous window's k-mer
        const uint32_t *wp = wbv + wbv_at(r, 0, mbM);
        for (uint32_t w0 = 0; w0 < m; w0 += 8) {
          // eight windows' minimizers loaded before any is used (one load in flight a lane kept
          // the kernel latency-bound: 6.9 ms at config 5)
          uint32_t pvs[8];
#pragma unroll
          for (int u = 0; u < 8; u++) pvs[u] = w0 + u < m ? wp[(uint64_t)(w0 + u) * 256u] : 0u;
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const uint32_t w = w0 + u;
            if (w >= m) break;
            const uint32_t pv = pvs[u];
            const bool open = w == 0 || pv != runv || runl == RUN_MAXW;
            runl = open ? 1u : runl + 1;
            runv = pv;
            myrec += open;
            if (open) {
                const uint32_t f = pv >> (32 - FINE_W_BITS);
                atomicAdd(&h_cnt[f >> 1], 1u << ((f & 1) * 16));  // overflow: checked after the group
            }
            if (((pv >> 12) & smask) == 0) {
                if (!have)
                    for (int t = 0; t < k; t++) roll_w(fwd, rc, code2(buf[s + w + t]), mask, sh);
                else
                    roll_w(fwd, rc, code2(buf[s + w + k - 1]), mask, sh);
                have = true;
                const K128 c = fwd < rc ? fwd : rc;
                const uint32_t hh = (uint32_t)(mix128(c) >> 32);
                const uint32_t j = hh >> (32 - HLL_REG_BITS);
                const uint32_t rho = (uint32_t)__clz((int)((hh << HLL_REG_BITS) | (1u << (HLL_REG_BITS - 1)))) + 1;
                if (rho > h_reg[j]) atomicMax(&h_reg[j], rho);
            } else {
                have = false;
            }
          }
        }
    }
    unsigned long long binsum = 0;  // bin-sum overflow check of k_upsweep
    __syncthreads();
    for (int i = threadIdx.x; i < FINE_W / 2; i += blockDim.x) binsum += (h_cnt[i] & 0xFFFFu) + (h_cnt[i] >> 16);
    for (int o = 32; o > 0; o >>= 1) {
        mypos += __shfl_down(mypos, o);
        myrec += __shfl_down(myrec, o);
        binsum += __shfl_down(binsum, o);
        mymax = max(mymax, (unsigned int)__shfl_down(mymax, o));
    }
    __shared__ unsigned long long s_diff;
    if (threadIdx.x == 0) s_diff = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_diff, myrec - binsum);
        if (mypos) atomicAdd(npos, mypos);
        if (mymax) atomicMax(maxlocal, mymax);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_diff != 0) atomicOr(skew, 1u);
    for (int i = threadIdx.x; i < FINE_W; i += blockDim.x) hist[g * FINE_W + i] = (h_cnt[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
    for (int i = threadIdx.x; i < (1 << HLL_REG_BITS); i += blockDim.x)
        hll_blocks[g * (1 << HLL_REG_BITS) + i] = (uint8_t)h_reg[i];
}

// ---- downsweep: records to their (coarse bucket, group) runs (count_part.h k_downsweep for
// clean reads, 24-B records, DS_RW windows per lane per round) -------------------------------
template <bool MB>
__global__ void __launch_bounds__(TILE_READS) k_downsweep_w(const uint8_t *buf, const uint64_t *off, uint64_t nreads,
                                                            int k, uint64_t gsize, uint64_t ngroups, int cbits,
                                                            const unsigned long long *offs, RecW *recs,
                                                            uint64_t read_base, const uint32_t *wbv, uint32_t mbM) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_W + 16];
    __shared__ RecW sorted[DS_BATCH_W];
    __shared__ uint8_t sbk[DS_BATCH_W];
    __shared__ unsigned int bcnt[1 << DS_MAX_CBITS], bbeg[1 << DS_MAX_CBITS];
    __shared__ unsigned long long cur[1 << DS_MAX_CBITS], gbase[1 << DS_MAX_CBITS];
    __shared__ unsigned int s_rounds, s_total, s_wave[TILE_READS / 64];
    const uint64_t g = blockIdx.x;
    const int C = 1 << cbits;
    const unsigned int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const K128 mask = kmask128(k);
    const int sh = 2 * (k - 1);
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
        stage_tile_w(buf, off, r0, r1, stage, base);  // fits: checked by the upsweep
        __syncthreads();
        const uint64_t r = r0 + tid;
        uint64_t s = 0, len = 0;
        if (r < r1) {
            s = off[r];
            len = off[r + 1] - s;
        }
        const uint32_t rel = (uint32_t)(s - base);
        const uint32_t m = len >= (uint64_t)k ? (uint32_t)(len - k + 1) : 0u;
        if (m) atomicMax(&s_rounds, (m + DS_RW - 1) / DS_RW);
        __syncthreads();
        const unsigned int nrounds = s_rounds;
        K128 fwd{0, 0}, rc{0, 0};
        uint32_t t = 0, w = 0;
        if (m)
            for (; t < (uint32_t)(k - 1); t++) roll_w(fwd, rc, code2(stage[rel + t]), mask, sh);
        const uint32_t m2 = 2 * m - 1;
        // MB: the round's minimizers are loaded one round ahead (a load per window right
        // before its use exposed its latency four times a round)
        uint32_t pvn[DS_RW];
        if (MB) {
#pragma unroll
            for (int j = 0; j < DS_RW; j++) pvn[j] = (uint32_t)j < m ? wbv[wbv_at(r, j, mbM)] : 0u;
        }
        for (unsigned int round = 0; round < nrounds; round++) {
            RecW rr[DS_RW];
            unsigned int cb[DS_RW], rk[DS_RW];
            uint32_t pvc[DS_RW];
            if (MB) {
#pragma unroll
                for (int j = 0; j < DS_RW; j++) {
                    pvc[j] = pvn[j];
                    const uint32_t wn = w + DS_RW + j;
                    pvn[j] = wn < m ? wbv[wbv_at(r, wn, mbM)] : 0u;
                }
            }
#pragma unroll
            for (int j = 0; j < DS_RW; j++) {
                cb[j] = 0xFFFFFFFFu;
                if (w < m) {
                    roll_w(fwd, rc, code2(stage[rel + t]), mask, sh);
                    const bool f = fwd < rc, pal = fwd == rc;
                    const K128 c = f ? fwd : rc;
                    uint32_t lC = f || pal ? w : m2 - w, lT = f && !pal ? m2 - w : w;
                    const uint32_t pv = MB ? pvc[j] : (uint32_t)(mix128(c) >> 32);
                    rr[j].lo = c.lo;
                    rr[j].hi = MB ? (c.hi | ((unsigned long long)(pv >> 8) << WMB_SHIFT)) : c.hi;
                    rr[j].read = (unsigned int)(r + read_base);
                    rr[j].ev = lC | (lT << 16);
                    cb[j] = cbits ? (pv >> (32 - cbits)) : 0u;
                    rk[j] = atomicAdd(&bcnt[cb[j]], 1u);
                    t++;
                    w++;
                }
            }
            __syncthreads();
            const unsigned int v = (int)tid < C ? bcnt[tid] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if ((int)lane >= o) incl += u;
            }
            if (lane == 63) s_wave[wid] = incl;
            __syncthreads();
            unsigned int before = 0;
            for (unsigned int q = 0; q < wid; q++) before += s_wave[q];
            if ((int)tid < C) {
                bbeg[tid] = before + incl - v;
                gbase[tid] = cur[tid];
                cur[tid] += v;
            }
            if (tid == TILE_READS - 1) s_total = before + incl;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < DS_RW; j++) {
                if (cb[j] != 0xFFFFFFFFu) {
                    const unsigned int p = bbeg[cb[j]] + rk[j];
                    sorted[p] = rr[j];
                    sbk[p] = (uint8_t)cb[j];
                }
            }
            __syncthreads();
            const unsigned int total = s_total;
            for (unsigned int i = tid; i < total; i += TILE_READS) {
                const unsigned int c = sbk[i];
                recs[gbase[c] + (i - bbeg[c])] = sorted[i];
            }
            if ((int)tid < C) bcnt[tid] = 0;
            __syncthreads();
        }
    }
}

// ---- downsweep of minimizer runs (RUNS): a lane's read closes a run where its minimizer
// changes (or the run holds RUN_MAXW windows) and at its last window; the runs go to their
// (coarse bucket, group) ranges through the same LDS counting sort as k_downsweep_w.  No read
// bytes are staged: a run needs only the window minimizers (k_wbv).
__global__ void __launch_bounds__(TILE_READS) k_downsweep_wr(const uint64_t *off, uint64_t nreads, int k,
                                                             uint64_t gsize, uint64_t ngroups, int cbits,
                                                             const unsigned long long *offs, RunWM *recs,
                                                             const uint32_t *wbv, uint32_t mbM) {
    constexpr int RW = DS_RW;
    constexpr int E = RW + 1;  // emissions a lane can make in a round (the last run closes extra)
    __shared__ RunWM sorted[TILE_READS * E];
    __shared__ uint8_t sbk[TILE_READS * E];
    __shared__ unsigned int bcnt[1 << DS_MAX_CBITS], bbeg[1 << DS_MAX_CBITS];
    __shared__ unsigned long long cur[1 << DS_MAX_CBITS], gbase[1 << DS_MAX_CBITS];
    __shared__ unsigned int s_rounds, s_total, s_wave[TILE_READS / 64];
    const uint64_t g = blockIdx.x;
    const int C = 1 << cbits;
    const unsigned int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t g0 = group_begin(g, gsize, nreads), g1 = group_begin(g + 1, gsize, nreads);
    for (uint64_t r0 = g0; r0 < g1; r0 += TILE_READS) {
        const uint64_t r1 = min(r0 + TILE_READS, g1);
        __syncthreads();
        for (int c = tid; c < C; c += TILE_READS) {
            if (r0 == g0) cur[c] = offs[(uint64_t)c * ngroups + g];
            bcnt[c] = 0;
        }
        if (tid == 0) s_rounds = 0;
        __syncthreads();
        const uint64_t r = r0 + tid;
        uint32_t m = 0;
        if (r < r1) {
            const uint64_t len = off[r + 1] - off[r];
            m = len >= (uint64_t)k ? (uint32_t)(len - k + 1) : 0u;
        }
        if (m) atomicMax(&s_rounds, (m + RW - 1) / RW);
        __syncthreads();
        const unsigned int nrounds = s_rounds;
        uint32_t w = 0, rs = 0, runv = 0;
        bool closed = m == 0;
        uint32_t pvn[RW];  // the next round's minimizers, loaded a round ahead
#pragma unroll
        for (int j = 0; j < RW; j++) pvn[j] = (uint32_t)j < m ? wbv[wbv_at(r, j, mbM)] : 0u;
        for (unsigned int round = 0; round < nrounds; round++) {
            RunWM rr[E];
            unsigned int cb[E], rk[E];
            uint32_t pvc[RW];
#pragma unroll
            for (int j = 0; j < RW; j++) {
                pvc[j] = pvn[j];
                const uint32_t wn = w + RW + j;
                pvn[j] = wn < m ? wbv[wbv_at(r, wn, mbM)] : 0u;
            }
            auto emit = [&](int j, uint32_t end) {  // the run [rs, end) of minimizer runv
                rr[j].read = (unsigned int)r;
                rr[j].wn = rs | ((end - rs) << 16);
                rr[j].place = runv >> 8;
                rr[j].pad = 0;
                cb[j] = cbits ? (runv >> (32 - cbits)) : 0u;
                rk[j] = atomicAdd(&bcnt[cb[j]], 1u);
            };
#pragma unroll
            for (int j = 0; j < E; j++) cb[j] = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < RW; j++) {
                if (w < m) {
                    const uint32_t pv = pvc[j];
                    if (w == 0) {
                        rs = 0;
                        runv = pv;
                    } else if (pv != runv || w - rs == RUN_MAXW) {
                        emit(j, w);
                        rs = w;
                        runv = pv;
                    }
                    w++;
                }
            }
            if (!closed && w == m) {
                emit(RW, m);
                closed = true;
            }
            __syncthreads();
            const unsigned int v = (int)tid < C ? bcnt[tid] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if ((int)lane >= o) incl += u;
            }
            if (lane == 63) s_wave[wid] = incl;
            __syncthreads();
            unsigned int before = 0;
            for (unsigned int q = 0; q < wid; q++) before += s_wave[q];
            if ((int)tid < C) {
                bbeg[tid] = before + incl - v;
                gbase[tid] = cur[tid];
                cur[tid] += v;
            }
            if (tid == TILE_READS - 1) s_total = before + incl;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < E; j++) {
                if (cb[j] != 0xFFFFFFFFu) {
                    const unsigned int p = bbeg[cb[j]] + rk[j];
                    sorted[p] = rr[j];
                    sbk[p] = (uint8_t)cb[j];
                }
            }
            __syncthreads();
            const unsigned int total = s_total;
            for (unsigned int i = tid; i < total; i += TILE_READS) {
                const unsigned int c = sbk[i];
                recs[gbase[c] + (i - bbeg[c])] = sorted[i];
            }
            if ((int)tid < C) bcnt[tid] = 0;
            __syncthreads();
        }
    }
}

// ---- third level, exact (round 4): fine bucket b's records split into its 2^sbits sub-buckets
// by two passes in one workgroup (LDS counts, then LDS cursors), written back to back from
// bstart[b]: b3[b 2^sbits + j] = first record of sub-bucket j.  The fixed-capacity regions of
// round 3 (mean + 30 % + 1024) assumed uniform hash buckets; minimizer buckets group whole
// minimizers (~(w + 1) / 2 k-mers x coverage records each), whose spread sent config-5-sized
// inputs past a few hundred sub-bucket capacities.  cap != 0 (tests): a sub-bucket past cap
// records raises *over, as the capacity did.
template <typename R>
__global__ void __launch_bounds__(512) k_split3(const R *in, const unsigned long long *bstart, int bbits, int sbits,
                                                R *out, unsigned long long *b3, unsigned long long cap,
                                                unsigned int *over) {
    __shared__ unsigned int cnt[64], cur[64];
    const unsigned int b = blockIdx.x, F = 1u << sbits, tid = threadIdx.x;
    const uint64_t r0 = bstart[b], r1 = bstart[b + 1];
    if (tid < 64) cnt[tid] = 0;
    __syncthreads();
    for (uint64_t i = r0 + tid; i < r1; i += 512) atomicAdd(&cnt[rec_bucket(in[i], bbits + sbits) & (F - 1)], 1u);
    __syncthreads();
    if (tid == 0) {
        unsigned int run = 0;
        for (unsigned int j = 0; j < F; j++) {
            cur[j] = run;
            b3[(uint64_t)b * F + j] = r0 + run;
            if (cap && cnt[j] > cap) *over = 1u;
            run += cnt[j];
        }
        if (b + 1 == gridDim.x) b3[(uint64_t)gridDim.x * F] = r1;
    }
    __syncthreads();
    for (uint64_t i = r0 + tid; i < r1; i += 512) {
        const R r = in[i];
        const unsigned int p = atomicAdd(&cur[rec_bucket(r, bbits + sbits) & (F - 1)], 1u);
        out[r0 + p] = r;
    }
}

// ---- minimizer runs back to window records (RUNS): after the refine, each fine bucket's runs
// are expanded into its windows' RecWM records -- split into the bucket's 2^sbits sub-buckets on
// the way (the third level; sbits = 0: one) -- so the bucket pass reads window records as before.
// Expanding inside the LDS-table kernel instead (one workgroup per table, a run's bases gathered
// as it rolls) took config 5's bucket pass from 16 to 70 ms: too few waves to hide the gathers.
struct RunReads {
    const uint8_t *buf;
    const uint64_t *off;
    int k;
    uint32_t m;          // windows per read (minimizer buckets: one read length)
    uint64_t read_base;  // global id of read 0
    const uint32_t *pk = nullptr;  // the reads as 2-bit codes (k_wbv, 16 a dword), pkd dwords a read
    uint32_t pkd = 0;
};
// windows per fine bucket (the expansion's output bases after a scan)
__global__ void __launch_bounds__(256) k_run_wsum(const RunWM *runs, const unsigned long long *bstart,
                                                  unsigned long long *wsum, uint64_t nb) {
    const uint64_t b = blockIdx.x;
    if (b >= nb) {  // (the scan's last element)
        if (threadIdx.x == 0) wsum[b] = 0;
        return;
    }
    unsigned long long w = 0;
    for (uint64_t i = bstart[b] + threadIdx.x; i < bstart[b + 1]; i += blockDim.x) w += runs[i].wn >> 16;
    for (int o = 32; o > 0; o >>= 1) w += __shfl_down(w, o);
    __shared__ unsigned long long s[4];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) wsum[b] = s[0] + s[1] + s[2] + s[3];
}
// fine bucket b's runs [bstart[b], bstart[b + 1]) -> out (same positions), sorted by their
// sub-bucket (the third level; sbits = 0: one); b3w[b 2^sbits + j] = first WINDOW record of
// sub-bucket j in the expansion's output (wstart[b] = the fine bucket's first)
__global__ void __launch_bounds__(512) k_split3_runs(const RunWM *in, const unsigned long long *bstart, int bbits,
                                                     int sbits, const unsigned long long *wstart, RunWM *out,
                                                     unsigned long long *b3w, unsigned long long cap,
                                                     unsigned int *over) {
    __shared__ unsigned int cnt[64], cur[64];
    __shared__ unsigned long long wc[64];
    const unsigned int b = blockIdx.x, F = 1u << sbits, tid = threadIdx.x;
    const uint64_t r0 = bstart[b], r1 = bstart[b + 1];
    if (tid < 64) cnt[tid] = 0, wc[tid] = 0;
    __syncthreads();
    for (uint64_t i = r0 + tid; i < r1; i += 512) {
        const RunWM x = in[i];
        const unsigned int j = rec_bucket(x, bbits + sbits) & (F - 1);
        atomicAdd(&cnt[j], 1u);
        atomicAdd(&wc[j], (unsigned long long)(x.wn >> 16));
    }
    __syncthreads();
    if (tid == 0) {
        unsigned int run = 0;
        unsigned long long w = wstart[b];
        for (unsigned int j = 0; j < F; j++) {
            cur[j] = run;
            b3w[(uint64_t)b * F + j] = w;
            if (cap && wc[j] > cap) *over = 1u;  // (tests: as k_split3's capacity)
            run += cnt[j];
            w += wc[j];
        }
        if (b + 1 == gridDim.x) b3w[(uint64_t)gridDim.x * F] = w;
    }
    __syncthreads();
    for (uint64_t i = r0 + tid; i < r1; i += 512) {
        const RunWM x = in[i];
        out[r0 + atomicAdd(&cur[rec_bucket(x, bbits + sbits) & (F - 1)], 1u)] = x;
    }
}

// fine bucket b's runs (in sub-bucket order) -> its windows' records at wstart[b] .., in run
// order: a workgroup takes the runs in batches, their window offsets scanned in LDS, and each
// thread a chunk of RUN_CHUNK consecutive windows -- its first run found by binary search, the
// k-mer rolled from the read's bases (RunReads), re-rolled where the chunk enters the next run.
// Consecutive threads write consecutive records, so a wave fills whole lines: with a lane per
// run, each lane wrote a stream of its own and the L2 evicted ~0.5 M open lines half written
// (27-39 ms at config 5, against ~10 ms here).
constexpr int RUN_BATCH = 2048;
constexpr int RUN_CHUNK = 16;
constexpr int RUN_DW = (RUN_CHUNK + WMB_MAX_K - 1 + 3 + 3) / 4;  // dwords a segment's bases span
static_assert(RUN_DW == 18, "segment dwords");
__global__ void __launch_bounds__(512) k_expand_runs(const RunWM *runs, const unsigned long long *bstart,
                                                     const unsigned long long *wstart, RecWM *out, RunReads rr) {
    __shared__ unsigned int pre[RUN_BATCH + 1];
    __shared__ unsigned int s_w[8];
    const unsigned int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t r0 = bstart[b], r1 = bstart[b + 1];
    const int k = rr.k;
    const K128 mask = kmask128(k);
    const int sh = 2 * (k - 1);
    const uint32_t m2 = 2 * rr.m - 1;
    uint64_t wout = wstart[b];
    for (uint64_t rb = r0; rb < r1; rb += RUN_BATCH) {
        const unsigned int nb = (unsigned int)min<uint64_t>(RUN_BATCH, r1 - rb);
        // window offsets of the batch's runs: 4 runs a thread, a block scan
        unsigned int v[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned int i = tid * 4 + u;
            v[u] = i < nb ? runs[rb + i].wn >> 16 : 0u;
            sum += v[u];
        }
        unsigned int incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int t = __shfl_up(incl, o);
            if ((int)lane >= o) incl += t;
        }
        if (lane == 63) s_w[wid] = incl;
        __syncthreads();
        unsigned int before = 0;
        for (unsigned int q = 0; q < wid; q++) before += s_w[q];
        unsigned int run = before + incl - sum;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned int i = tid * 4 + u;
            if (i < nb) pre[i] = run;
            run += v[u];
        }
        if (tid == 511) pre[nb] = run;  // (tid 511's run is the batch total: nb <= 4 * 512)
        __syncthreads();
        const unsigned int W = pre[nb];
        for (unsigned int q0 = tid * RUN_CHUNK; q0 < W; q0 += 512 * RUN_CHUNK) {
            const unsigned int q1 = min(q0 + RUN_CHUNK, W);
            unsigned int lo = 0, hi = nb;  // the run holding window q0: pre[lo] <= q0 < pre[lo + 1]
            while (hi - lo > 1) {
                const unsigned int md = (lo + hi) >> 1;
                if (pre[md] <= q0) lo = md;
                else hi = md;
            }
            unsigned int i = lo, j = q0 - pre[lo];
            // segments: the chunk's windows within one run -- their n + k - 1 bases loaded as
            // dwords at once (RUN_DW of them: k <= WMB_MAX_K), the byte steps unrolled over
            // registers (a load per base left each step waiting on its latency: 85 ms at config 5)
            for (unsigned int q = q0; q < q1;) {
                const RunWM x = runs[rb + i];
                const uint32_t ws = x.wn & 0xFFFFu, n = x.wn >> 16;
                const uint32_t cnt = min(n - j, q1 - q);
                const uint64_t s0 = rr.off[x.read] + ws + j;
                const uint32_t skip = (uint32_t)(s0 & 3), nbytes = cnt + (uint32_t)k - 1;
                const uint32_t nw = (skip + nbytes + 3) >> 2;
                const uint32_t *wp = reinterpret_cast<const uint32_t *>(rr.buf + (s0 & ~3ull));
                uint32_t d[RUN_DW];
#pragma unroll
                for (int u = 0; u < RUN_DW; u++) d[u] = (uint32_t)u < nw ? wp[u] : 0u;
                const unsigned int rd = (unsigned int)(rr.read_base + x.read);
                const unsigned long long pbits = (unsigned long long)x.place << WMB_SHIFT;
                RecWM *o = out + wout + q;
                K128 fwd{0, 0}, rc{0, 0};
#pragma unroll
                for (int u = 0; u < RUN_DW; u++) {
#pragma unroll
                    for (int bt = 0; bt < 4; bt++) {
                        const uint32_t bpos = (uint32_t)(u * 4 + bt);
                        if (bpos < skip || bpos >= skip + nbytes) continue;
                        roll_w(fwd, rc, code2((d[u] >> (8 * bt)) & 0xFFu), mask, sh);
                        const uint32_t tt = bpos - skip;
                        if (tt + 1 < (uint32_t)k) continue;
                        const uint32_t jj = tt + 1 - (uint32_t)k, w = ws + j + jj;
                        const bool f = fwd < rc, pal = fwd == rc;
                        const K128 c = f ? fwd : rc;
                        const uint32_t lC = f || pal ? w : m2 - w, lT = f && !pal ? m2 - w : w;
                        RecWM r;
                        r.lo = c.lo;
                        r.hi = c.hi | pbits;
                        r.read = rd;
                        r.ev = lC | (lT << 16);
                        o[jj] = r;
                    }
                }
                q += cnt;
                j += cnt;
                if (j == n) i++, j = 0;
            }
        }
        wout += W;
        __syncthreads();  // (pre is rewritten by the next batch)
    }
}

// ---- bucket pass: one LDS table of 128-bit keys per final bucket ----------------------------
// Slots claim a key with two 64-bit CASes on its claim words (wide_w1 / wide_w2, never 0),
// as wide_slot does in HBM; a slot whose first word matches but whose second word went to
// another key is passed over.  Wave-uniform probe loop and fill reservation as lds_insert.
struct alignas(16) LSlotW {
    unsigned long long w1, w2;
    unsigned int count, pad;
    unsigned long long fC, fT;  // fC, fT 16-B aligned
    unsigned long long pad2;
};
static_assert(sizeof(LSlotW) == 48, "wide LDS slot layout");

// table sizes need not be powers of two: slot0 = (low 32 hash bits * SLOTS) >> 32
__host__ __device__ inline unsigned int wide_slot0(uint64_t h, unsigned int slots) {
    return (unsigned int)(((uint64_t)(uint32_t)h * slots) >> 32);
}

// k_bucket_wr's slot (round 6): LSlotW without its padding, 40 B -- 1664 slots in 65 KB, so with
// 512 threads and a 1024-dword code stage two workgroups share a CU's 160 KB (one at 104 KB)
struct LSlotW40 {
    unsigned long long w1, w2;
    unsigned int count, pad;
    unsigned long long fC, fT;
};
static_assert(sizeof(LSlotW40) == 40, "compact wide LDS slot layout");

template <int SLOTS, typename Slot = LSlotW>
__device__ inline void lds_insert_w(Slot *tab, unsigned int *s_over, const K128 &c, unsigned int slot0,
                                    unsigned int add, unsigned long long eC, unsigned long long eT) {
    const unsigned long long w1 = wide_w1(c), w2 = wide_w2(c);
    unsigned int slot = slot0;
    unsigned long long a = tab[slot].w1, bw = tab[slot].w2;
    bool miss = !(a == w1 && bw == w2);
#pragma unroll 1
    while (__any(miss)) {
        if (miss) {
            if (a == 0) {  // free slot: reserve, then claim the first word
                if (atomicAdd(&s_over[1], 1u) >= SLOTS - 1) {
                    s_over[0] = 1;
                    a = w1;
                    bw = w2;  // give up (the bucket is redone elsewhere)
                } else {
                    a = atomicCAS(&tab[slot].w1, 0ull, w1);
                    if (a == 0) a = w1;
                    else atomicSub(&s_over[1], 1u);
                }
            }
            if (a == w1 && bw != w2) {  // first word ours: the second decides
                bw = tab[slot].w2;
                if (bw == 0) {
                    bw = atomicCAS(&tab[slot].w2, 0ull, w2);
                    if (bw == 0) bw = w2;
                }
            }
            if (!(a == w1 && bw == w2)) {
                slot = slot + 1 == SLOTS ? 0u : slot + 1;
                a = tab[slot].w1;
                bw = tab[slot].w2;
            }
            miss = !(a == w1 && bw == w2);
        }
    }
    Slot &sl = tab[slot];
    atomicAdd(&sl.count, add);
    ulonglong2 ev;
    if constexpr (sizeof(Slot) % 16 == 0) ev = *reinterpret_cast<const ulonglong2 *>(&sl.fC);  // (16-B aligned)
    else ev = make_ulonglong2(sl.fC, sl.fT);
    if (eC < ev.x) atomicMin(&sl.fC, eC);
    if (eT < ev.y) atomicMin(&sl.fT, eT);
}

// ---- bucket pass on minimizer runs (RUNS, third level) ------------------------------------------
// One workgroup per table as k_bucket_w, but the table's records are its RUNS (k_split3<RunWM>:
// sorted by sub-bucket, bounds in run units): their bases are gathered once into LDS as 2-bit
// codes (a thread a run, 16 bases a dword), then every window of the table is a thread's -- its
// run by binary search over the window offsets, its k-mer extracted from the codes (the reverse
// complement is ~codes, the forward string its twin) -- and inserted.  The window records never
// exist: config 5's expansion wrote and the bucket pass read back 30 GB of them (29 + 16 ms).
constexpr int WR_NT = 1024;        // threads a table (one workgroup per CU: 104 KB of LDS)
constexpr int WR_CODES = 2048;     // code dwords a batch of runs stages (32 K bases)
__device__ inline K128 extract_codes(const uint32_t *c, uint32_t bitpos) {  // bits [bitpos, bitpos + 128)
    const uint32_t w = bitpos >> 5, sft = bitpos & 31;
    uint32_t d[5];
#pragma unroll
    for (int u = 0; u < 5; u++) d[u] = c[w + u];
    uint32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; u++) o[u] = sft ? __builtin_amdgcn_alignbit(d[u + 1], d[u], sft) : d[u];
    return K128{(unsigned long long)o[0] | (unsigned long long)o[1] << 32, (unsigned long long)o[2] | (unsigned long long)o[3] << 32};
}
// the runs' bases as 2-bit codes in global memory, run after run in their (sub-bucket sorted)
// order: per fine bucket b its code dwords (k_run_ccount, scanned -> cbase[b]), then each run's
// codes at cbase[b] + the prefix of its fine bucket's runs (k_run_codes: a thread a run, all
// lanes busy, the gathers' latency hidden by full occupancy); ctab[t] = first code dword of
// table t (sub-bucket bounds b3 in run units).  The bucket pass then loads a table's codes as
// one contiguous block -- gathering them itself, one workgroup per CU, it waited on them
// (k_bucket_wr 55 ms at config 5).
__device__ inline unsigned int run_cdw(const RunWM &x, int k) { return ((x.wn >> 16) + (unsigned int)k - 1 + 15) >> 4; }
__global__ void __launch_bounds__(256) k_run_ccount(const RunWM *runs, const unsigned long long *bstart, int k,
                                                    unsigned long long *csum, uint64_t nb) {
    const uint64_t b = blockIdx.x;
    if (b >= nb) {
        if (threadIdx.x == 0) csum[b] = 0;
        return;
    }
    unsigned long long c = 0;
    for (uint64_t i = bstart[b] + threadIdx.x; i < bstart[b + 1]; i += blockDim.x) c += run_cdw(runs[i], k);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
    __shared__ unsigned long long sm[4];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) csum[b] = sm[0] + sm[1] + sm[2] + sm[3];
}
__global__ void __launch_bounds__(512) k_run_codes(const RunWM *runs, const unsigned long long *bstart,
                                                   const unsigned long long *cbase, const unsigned long long *b3, int sbits,
                                                   uint32_t *codes, unsigned long long *ctab, RunReads rr) {
    __shared__ unsigned int s_w[8];
    __shared__ unsigned long long s_off;
    const unsigned int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, F = 1u << sbits;
    const uint64_t r0 = bstart[b], r1 = bstart[b + 1];
    const int k = rr.k;
    if (tid == 0) s_off = cbase[b];
    __syncthreads();
    for (uint64_t rb = r0; rb < r1; rb += 512) {
        const uint64_t ri = rb + tid;
        RunWM x{};
        unsigned int nc = 0;
        if (ri < r1) x = runs[ri], nc = run_cdw(x, k);
        unsigned int incl = nc;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int t = __shfl_up(incl, o);
            if ((int)lane >= o) incl += t;
        }
        if (lane == 63) s_w[wid] = incl;
        __syncthreads();
        unsigned int before = 0, tot = 0;
        for (unsigned int q = 0; q < 8; q++) {
            if (q < wid) before += s_w[q];
            tot += s_w[q];
        }
        const unsigned long long od0 = s_off + before + incl - nc;
        if (ri < r1) {
            // a table's first run: its code base (the sub-bucket bounds are runs of this bucket)
            for (unsigned int j = 0; j < F; j++)
                if (b3[(uint64_t)b * F + j] == ri) ctab[(uint64_t)b * F + j] = od0;
            const unsigned int nwin = x.wn >> 16, nbases = nwin + (unsigned int)k - 1;
            if (rr.pk) {  // from k_wbv's 2-bit reads: a shifted copy of the read's code dwords
                const uint32_t *pr = rr.pk + (uint64_t)x.read * rr.pkd;
                const unsigned int st = x.wn & 0xFFFFu, q0 = st >> 4, sft = 2 * (st & 15), ncd = run_cdw(x, k);
                for (unsigned int q = 0; q < ncd; q++) {
                    const uint32_t lo = pr[q0 + q], hi = q0 + q + 1 < rr.pkd ? pr[q0 + q + 1] : 0u;
                    uint32_t v = sft ? __builtin_amdgcn_alignbit(hi, lo, sft) : lo;
                    const unsigned int rem = nbases - 16 * q;  // (the run's last dword: its bases only)
                    if (rem < 16) v &= (1u << (2 * rem)) - 1u;
                    codes[od0 + q] = v;
                }
            } else {
                const uint64_t s0 = rr.off[x.read] + (x.wn & 0xFFFFu);
                const uint32_t *wp = reinterpret_cast<const uint32_t *>(rr.buf + (s0 & ~3ull));
                const unsigned int skip = (unsigned int)(s0 & 3), nw = (skip + nbases + 3) >> 2;
                uint32_t acc = 0;
                unsigned int i = 0;
                unsigned long long od = od0;
                for (unsigned int q = 0; q < nw; q += 8) {
                    uint32_t d[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) d[u] = q + u < nw ? wp[q + u] : 0u;
#pragma unroll
                    for (int u = 0; u < 8; u++)
#pragma unroll
                        for (int bt = 0; bt < 4; bt++) {
                            const unsigned int bp = (q + u) * 4 + bt;
                            if (bp < skip || bp >= skip + nbases) continue;
                            acc |= code2((d[u] >> (8 * bt)) & 0xFFu) << (2 * (i & 15));
                            if ((i & 15) == 15) codes[od++] = acc, acc = 0;
                            i++;
                        }
                }
                if (i & 15) codes[od] = acc;
            }
        }
        __syncthreads();
        if (tid == 0) s_off += tot;
        __syncthreads();
    }
    if (tid == 0 && b + 1 == gridDim.x) ctab[(uint64_t)gridDim.x * F] = s_off;
}

template <int SLOTS, int NT, typename Slot = LSlotW>
__device__ inline void bucket_w_finish(const Slot *tab, unsigned int b, long long limit, K128 *dkey, unsigned int *dcnt,
                                       unsigned long long *dfc, unsigned long long *dft, SubSlotW *sub,
                                       unsigned int *nsolid, unsigned long long *ndistinct, unsigned int *bmark,
                                       unsigned int *s_wave, unsigned int *s_pres, unsigned int &s_base);

// (WR_NT / WR_CODES / LSlotW: one 104-KB workgroup per CU, round 5; NT = 512, CODES = 1024,
// LSlotW40: two 79-KB workgroups per CU, round 6)
template <int SLOTS, int WR_NT = ::ec::WR_NT, int WR_CODES = ::ec::WR_CODES, typename Slot = LSlotW>
__global__ void __launch_bounds__(WR_NT) k_bucket_wr(const RunWM *runs, const unsigned long long *bstart,
                                                    const unsigned long long *bend, long long limit, K128 *dkey,
                                                    unsigned int *dcnt, unsigned long long *dfc, unsigned long long *dft,
                                                    SubSlotW *sub, unsigned int *nsolid, unsigned long long *ndistinct,
                                                    unsigned int *overflow, unsigned int *bmark, RunReads rr,
                                                    const uint32_t *gcodes, const unsigned long long *ctab) {
    __shared__ Slot tab[SLOTS];
    __shared__ unsigned int s_over[2];
    __shared__ unsigned int s_wave[WR_NT / 64], s_pres[WR_NT / 64], s_wave2[WR_NT / 64];
    __shared__ unsigned int s_base, s_nb;
    __shared__ unsigned int wpre[WR_NT + 1], cpre[WR_NT + 1];  // window / code-dword offsets of the batch's runs
    __shared__ uint2 rmeta[WR_NT];                              // read, first window
    __shared__ uint32_t codes[WR_CODES + 8];
    const unsigned int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int i = tid; i < SLOTS; i += WR_NT) {
        tab[i].w1 = 0;
        tab[i].w2 = 0;
        tab[i].count = 0;
        tab[i].fC = NONE64;
        tab[i].fT = NONE64;
    }
    if (tid == 0) s_over[0] = 0, s_over[1] = 0;
    __syncthreads();
    const uint64_t r0 = bstart[b], r1 = bend ? bend[b] : bstart[b + 1];
    const int k = rr.k;
    const K128 mask = kmask128(k);
    const uint32_t m2 = 2 * rr.m - 1;
    unsigned long long gco = ctab[b];  // the batch's first code dword in gcodes
    for (uint64_t rb = r0; rb < r1;) {
        // the batch: up to WR_NT runs whose codes fit WR_CODES dwords (a run of n windows: n + k - 1 bases)
        const uint64_t ri = rb + tid;
        RunWM x{};
        unsigned int nwin = 0, ncd = 0;
        if (ri < r1) {
            x = runs[ri];
            nwin = x.wn >> 16;
            ncd = (nwin + (unsigned int)k - 1 + 15) >> 4;
        }
        // two block scans at once (windows, code dwords)
        unsigned int iw = nwin, ic = ncd;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int tw = __shfl_up(iw, o), tc = __shfl_up(ic, o);
            if ((int)lane >= o) iw += tw, ic += tc;
        }
        if (lane == 63) s_wave[wid] = iw, s_wave2[wid] = ic;
        __syncthreads();
        unsigned int bw = 0, bc = 0;
        for (unsigned int q = 0; q < wid; q++) bw += s_wave[q], bc += s_wave2[q];
        const unsigned int cw = bw + iw - nwin, cc = bc + ic - ncd;  // exclusive offsets
        const bool in = ri < r1 && cc + ncd <= WR_CODES;             // (runs past the codes wait for the next batch)
        if (tid == 0) s_nb = 0;
        __syncthreads();
        if (in) atomicMax(&s_nb, tid + 1);  // (a prefix: offsets grow with tid)
        __syncthreads();
        const unsigned int nb = s_nb;
        if (tid < nb) {
            wpre[tid] = cw;
            cpre[tid] = cc;
            rmeta[tid] = make_uint2(x.read, x.wn & 0xFFFFu);
            if (tid + 1 == nb) wpre[nb] = cw + nwin, cpre[nb] = cc + ncd;
        }
        __syncthreads();
        // the batch's codes: one contiguous block of gcodes (k_run_codes)
        const unsigned int ncodes = cpre[nb];
        for (unsigned int i = tid; i < ncodes; i += WR_NT) codes[i] = gcodes[gco + i];
        gco += ncodes;
        __syncthreads();
        // the batch's windows, a thread each
        const unsigned int W = wpre[nb];
        for (unsigned int q = tid; q < W; q += WR_NT) {
            unsigned int lo = 0, hi = nb;
            while (hi - lo > 1) {
                const unsigned int md = (lo + hi) >> 1;
                if (wpre[md] <= q) lo = md;
                else hi = md;
            }
            const unsigned int j = q - wpre[lo];
            const uint2 mt = rmeta[lo];
            const K128 V = extract_codes(codes, cpre[lo] * 32 + 2 * j);  // bases j .., first least significant
            const K128 rc{~V.lo & mask.lo, ~V.hi & mask.hi};
            const K128 fwd = twin128(rc, k);
            const uint32_t w = mt.y + j;
            const bool f = fwd < rc, pal = fwd == rc;
            const K128 c = f ? fwd : rc;
            const uint32_t lC = f || pal ? w : m2 - w, lT = f && !pal ? m2 - w : w;
            const unsigned long long rd = (unsigned long long)(rr.read_base + mt.x) << 32;
            lds_insert_w<SLOTS, Slot>(tab, s_over, c, wide_slot0(mix128(c), SLOTS), lC == lT ? 2u : 1u, rd | lC,
                                      rd | lT);
        }
        rb += nb;
        if (nb == 0) {  // (one run past WR_CODES: never for k <= 52 and reads <= 160 bp -- reported)
            if (tid == 0) s_over[0] = 1;
            __syncthreads();
            break;
        }
        __syncthreads();  // (the batch's staging is rewritten by the next)
    }
    if (s_over[0]) {
        if (tid == 0) atomicAdd(overflow, 1u);
        return;
    }
    bucket_w_finish<SLOTS, WR_NT, Slot>(tab, b, limit, dkey, dcnt, dfc, dft, sub, nsolid, ndistinct, bmark, s_wave,
                                        s_pres, s_base);
}

// ---- third partition level (more keys than 2^FINE_W_BITS tables hold) ---------------------
// The upsweep's fine histogram sizes 2^FINE_W_BITS buckets exactly; past ~1.8e7 distinct keys
// each of them is split again by the next hash bits into 2^s sub-buckets of fixed capacity
// (k_refine with fcap: the hash is uniform, so a sub-bucket holds its mean +- a few sigma).
// bstart3[c << s] = bstart[c] gives k_refine its input ranges; cursors start at d * fcap.
__global__ void __launch_bounds__(256) k_level3_init(const unsigned long long *bstart, uint64_t nfine, int s,
                                                     uint64_t fcap, unsigned long long *bstart3,
                                                     unsigned long long *gcur) {
    const uint64_t F = 1ull << s;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t <= nfine * F;
         t += (uint64_t)gridDim.x * blockDim.x) {
        if ((t & (F - 1)) == 0) bstart3[t] = bstart[t >> s];
        if (t < nfine * F) gcur[t] = t * fcap;
    }
}
// bucket d's records: [d * fcap, min(gcur[d], (d + 1) * fcap))
__global__ void __launch_bounds__(256) k_level3_ends(const unsigned long long *gcur, uint64_t nb, uint64_t fcap,
                                                     unsigned long long *bbeg, unsigned long long *bend) {
    for (uint64_t d = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; d < nb; d += (uint64_t)gridDim.x * blockDim.x) {
        bbeg[d] = d * fcap;
        bend[d] = min((uint64_t)gcur[d], (d + 1) * fcap);
    }
}

// solid filter + compaction of a filled table (as lds_table_finish): the solid keys to the
// dense arrays at a block-reserved base, the slots to the bucket's sub-table region
template <int SLOTS, int NT, typename Slot>
__device__ inline void bucket_w_finish(const Slot *tab, unsigned int b, long long limit, K128 *dkey, unsigned int *dcnt,
                                       unsigned long long *dfc, unsigned long long *dft, SubSlotW *sub,
                                       unsigned int *nsolid, unsigned long long *ndistinct, unsigned int *bmark,
                                       unsigned int *s_wave, unsigned int *s_pres, unsigned int &s_base) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int PER = (SLOTS + NT - 1) / NT;
    bool solid[PER];
    unsigned int mine = 0, present = 0;
    for (int q = 0; q < PER; q++) {
        const int idx = threadIdx.x * PER + q;
        if (idx >= SLOTS) {
            solid[q] = false;
            continue;
        }
        const Slot &sl = tab[idx];
        present += sl.w1 != 0;
        solid[q] = sl.w1 != 0 && (long long)sl.count > limit;
        mine += solid[q];
    }
    unsigned int incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) s_wave[wid] = incl;
    unsigned int pres = present;
    for (int o = 32; o > 0; o >>= 1) pres += __shfl_down(pres, o);
    if (lane == 0) s_pres[wid] = pres;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned int tot = 0, np = 0;
        for (int w = 0; w < NT / 64; w++) {
            const unsigned int c = s_wave[w];
            s_wave[w] = tot;
            tot += c;
            np += s_pres[w];
        }
        s_base = tot ? atomicAdd(nsolid, tot) : 0;
        if (np) atomicAdd(ndistinct, (unsigned long long)np);
        if (bmark && tot) atomicOr(&bmark[s_base >> 5], 1u << (s_base & 31));  // (the tile ranking's cuts)
    }
    __syncthreads();
    unsigned int u = s_base + s_wave[wid] + incl - mine;
    SubSlotW *region = sub ? sub + (uint64_t)b * SLOTS : nullptr;
    for (int q = 0; q < PER; q++) {
        const int idx = threadIdx.x * PER + q;
        if (idx >= SLOTS) break;
        const Slot &sl = tab[idx];
        SubSlotW o;
        o.w1 = sl.w1;
        o.w2 = sl.w2;
        o.id = NONE32;
        o.pad = 0;
        o.pad2 = 0;
        if (solid[q]) {
            dkey[u] = wide_key(sl.w1, sl.w2);
            dcnt[u] = sl.count;
            dfc[u] = sl.fC;
            dft[u] = sl.fT;
            o.id = u;
            u++;
        }
        if (region) region[idx] = o;
    }
}

// bend != nullptr: bucket b is [bstart[b], bend[b]) (third level), else [bstart[b], bstart[b + 1])
template <int SLOTS, typename R = RecW>
__global__ void __launch_bounds__(BUCKET_THREADS) k_bucket_w(const R *recs, const unsigned long long *bstart,
                                                            const unsigned long long *bend, long long limit, K128 *dkey, unsigned int *dcnt,
                                                            unsigned long long *dfc, unsigned long long *dft,
                                                            SubSlotW *sub, unsigned int *nsolid,
                                                            unsigned long long *ndistinct, unsigned int *overflow,
                                                            unsigned int *bmark = nullptr) {
    __shared__ LSlotW tab[SLOTS];
    __shared__ unsigned int s_over[2];
    __shared__ unsigned int s_wave[BUCKET_THREADS / 64], s_pres[BUCKET_THREADS / 64];
    __shared__ unsigned int s_base;
    const unsigned int b = blockIdx.x;
    for (int i = threadIdx.x; i < SLOTS; i += blockDim.x) {
        tab[i].w1 = 0;
        tab[i].w2 = 0;
        tab[i].count = 0;
        tab[i].fC = NONE64;
        tab[i].fT = NONE64;
    }
    if (threadIdx.x == 0) {
        s_over[0] = 0;
        s_over[1] = 0;
    }
    __syncthreads();
    const uint64_t r0 = bstart[b], r1 = bend ? bend[b] : bstart[b + 1];
    {
        constexpr int U = 4;  // loads of U records issued before any insert
        auto ins = [&](const R &x) {
            const unsigned int lC = x.ev & 0xFFFFu, lT = x.ev >> 16;
            const K128 c = rkey(x);
            const unsigned long long rd = (unsigned long long)x.read << 32;
            lds_insert_w<SLOTS>(tab, s_over, c, wide_slot0(mix128(c), SLOTS), lC == lT ? 2u : 1u, rd | lC, rd | lT);
        };
        uint64_t i = r0 + threadIdx.x;
        for (; i + (U - 1) * (uint64_t)blockDim.x < r1; i += U * (uint64_t)blockDim.x) {
            R raw[U];
#pragma unroll
            for (int u = 0; u < U; u++) raw[u] = recs[i + u * (uint64_t)blockDim.x];
#pragma unroll
            for (int u = 0; u < U; u++) ins(raw[u]);
        }
        for (; i < r1; i += blockDim.x) ins(recs[i]);
    }
    __syncthreads();
    if (s_over[0]) {
        if (threadIdx.x == 0) atomicAdd(overflow, 1u);
        return;
    }
    bucket_w_finish<SLOTS, BUCKET_THREADS>(tab, b, limit, dkey, dcnt, dfc, dft, sub, nsolid, ndistinct, bmark, s_wave,
                                           s_pres, s_base);
}

}  // namespace ec
