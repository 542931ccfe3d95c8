// count_sk2.h -- super-k-mer records on the count_v2 scaffold (N-free reads of one length,
// 21 <= k <= 32).
//
// count_v2.h moves one 10- or 12-byte record per k-mer position through partition, refine
// and bucket: ~30 GB of HBM traffic at the headline size.  Consecutive windows of a read that
// share their minimizer (superkmer.h: the smallest hash over the window's canonical m-mers,
// the same for a k-mer and its twin) form a super-k-mer; all its k-mers belong to the
// minimizer's bucket, so the run travels as ONE 16-byte record holding its L = n + k - 1
// bases (2 bits each, n <= 16 windows) -- about (w + 1) / 2 windows per record:
//
//   k_skpart    per read group : lane = read; m-mer hashes and van Herk / Gil-Werman sliding
//                                minima (block length w, LDS ring), runs of equal minimizer
//                                buffered as 4-byte entries (read lane, first window, n,
//                                bucket bits); a flush sorts the wave's entries by coarse
//                                bucket and writes 16-byte records to the (group, coarse)
//                                runs, bases read back from the wave's 2-bit stage;
//                                HyperLogLog of the k-mers of sampled minimizers
//   k_skrefine  per coarse slice: runs -> fixed-capacity final buckets (as k_refine2), the
//                                group-relative position made absolute
//   k_skbucket  per final bucket: records sorted by window count in LDS, lane = record, the
//                                k-mers rolled out of the bases into the LDS table of
//                                count_part.h (lds_insert / lds_table_finish)
//   SolidIndex (graph.h, sk = 1): a key's bucket = the top bits of min_remix(its minimizer),
//                                first probe slot = sk_slot(key) -- as k_bucket_sk wrote them
//
// Record (uint4): x, y = bases 0..15, 16..31 (base i at bits 2i), z = bases 32..45 in bits
// 0..27 | (n - 1) << 28; w = partition: bucket-bits-below-coarse (8) << 24 | p_rel (24 bits,
// (read - g0) * M + first window); refine output: p = (read_base + read) * M + first window.
// Events as count_part.h: read = p / M, lf = p % M + o for window o, lr = 2M - 1 - lf.
#pragma once
#include "count_v2.h"
#include "superkmer.h"

namespace ec {

constexpr int SK2_NMAX = 16;     // windows per record (n - 1 in 4 bits)
// entries a partition wave buffers: 1024 (40 KB of LDS a workgroup at NPF = 7: four workgroups,
// four waves a SIMD, per CU).  A round adds ~2 W / (W + 1) entries a lane (~114 a wave at
// k = 31), at most 64 W: the buffer is flushed past SK2_FLUSH_AT, which leaves room for 10 entries
// a lane in the next round; a round that outgrows even that (never on sequence data: every lane's
// minimizer changing at almost every window) stops storing and sets *overflow (the call is
// redone on window records)
constexpr int SK2_ECAP_W = 1024;
constexpr int SK2_FLUSH_AT = SK2_ECAP_W - 64 - 640;
#ifndef SK2_PD_DEF
#define SK2_PD_DEF 4
#endif
constexpr int SK2_PD = SK2_PD_DEF;  // k_skbucket record rounds in flight per thread
constexpr int SK2_HQ = 128;      // sampled runs a partition wave queues for the HyperLogLog
constexpr int SK2_BASES = 46;    // bases per record (92 bits)
#ifndef SK2_TILE_DEF
#define SK2_TILE_DEF 2048
#endif
constexpr int SK2_TILE = SK2_TILE_DEF;  // k_skrefine records per tile (A/B: 2048 0.70 ms, 4096 0.81, 8192 0.85)
constexpr int SK2_CBITS = 6;     // coarse buckets of the partition: 64
constexpr int SK2_BBITS = 14;    // final buckets <= 2^14 (bucket bits in an entry)
constexpr int SK2_FBITS = SK2_BBITS - SK2_CBITS;  // bucket bits below the coarse bits in a record

__host__ __device__ constexpr inline uint32_t sk2_nmax(int k) {
    return (uint32_t)(SK2_BASES - k + 1 < SK2_NMAX ? SK2_BASES - k + 1 : SK2_NMAX);
}

// ---- partition -------------------------------------------------------------------------------
// A wave's flush: its cntw buffered entries counting-sorted by coarse bucket (the wave's own
// counters, DPP scan), each bucket's run reserved on the workgroup cursor (spill records past
// the capacity), the 16-B records built from the wave's 2-bit stage and stored as runs.
__device__ inline uint32_t sk_bases16(const uint32_t *st, uint32_t p) {
    return __builtin_amdgcn_alignbit(st[(p >> 4) + 1], st[p >> 4], 2 * (p & 15));
}
// u8 HyperLogLog register max by CAS on the word holding it
__device__ inline void sk_hll_put(unsigned int *s_hll, uint32_t hh) {
    const uint32_t hj = hh >> (32 - HLL_REG_BITS);
    const uint32_t rho = (uint32_t)__clz((int)((hh << HLL_REG_BITS) | (1u << (HLL_REG_BITS - 1)))) + 1;
    const uint32_t hs = (hj & 3) * 8;
    uint32_t old = s_hll[hj >> 2];
    while (rho > ((old >> hs) & 0xFFu)) {
        const uint32_t nw = (old & ~(0xFFu << hs)) | (rho << hs);
        const uint32_t prev = atomicCAS(&s_hll[hj >> 2], old, nw);
        if (prev == old) break;
        old = prev;
    }
}

template <int C>
__device__ inline void skpart_flush(uint32_t cntw, const uint32_t *ent, uint16_t *srt, unsigned int *wcnt,
                                    unsigned int *cur, unsigned long long *base, const uint32_t *rel,
                                    const uint32_t *st, uint32_t lane, unsigned long long gcap, uint64_t cap,
                                    unsigned long long spill, uint32_t M, uint32_t rtile, uint4 *recs,
                                    unsigned int *overflow, unsigned int *s_hll, uint32_t *hq, uint32_t smaskb,
                                    int k, uint64_t kmask) {
    wave_sync();
    for (uint32_t i = lane; i < cntw; i += 64) atomicAdd(&wcnt[ent[i] >> 26], 1u);
    wave_sync();
    const unsigned int v = lane < (uint32_t)C ? wcnt[lane] : 0u;
    const unsigned int incl = wave_incl_scan(v);
    const unsigned int beg = incl - v;
    if (lane < (uint32_t)C) {
        wcnt[lane] = beg;
        unsigned int at = 0;
        if (v) at = atomicAdd(&cur[lane], v);
        unsigned long long b0 = gcap + lane * cap + at - beg;
        if (at + v > cap) {  // past the capacity: stores go to the spill records
            atomicOr(overflow, 1u);
            b0 = spill - beg;
        }
        base[lane] = b0;
    }
    wave_sync();
    for (uint32_t i = lane; i < cntw; i += 64) {
        const unsigned int p = atomicAdd(&wcnt[ent[i] >> 26], 1u);
        srt[p] = (uint16_t)i;
    }
    wave_sync();
    // HyperLogLog over the k-mers of the runs whose minimizer's low bucket bits & smaskb are 0 (a
    // sample of minimizer space; a k-mer and its twin share the minimizer): sampled runs are
    // queued (stage position | (n - 1) << 16) and their windows spread over the lanes when the
    // queue fills -- a per-lane loop over its run's windows held the whole wave whenever one
    // lane of 64 had a sampled run
    uint32_t nq = 0;  // (uniform)
    auto hll_drain = [&]() {
        wave_sync();
        for (uint32_t x = lane; x < nq * SK2_NMAX; x += 64) {
            const uint32_t qe = hq[x / SK2_NMAX], q = x % SK2_NMAX;
            if (q <= (qe >> 16)) {
                const uint32_t p = (qe & 0xFFFFu) + q;
                const uint64_t K = (uint64_t)sk_bases16(st, p) | (uint64_t)sk_bases16(st, p + 16) << 32;
                const uint64_t krc = ~K & kmask, kfw = rev2_64(K) >> (64 - 2 * k);
                sk_hll_put(s_hll, (uint32_t)(mix64(kfw < krc ? kfw : krc) >> 32));
            }
        }
        wave_sync();
        nq = 0;
    };
    for (uint32_t i0 = 0; i0 < cntw; i0 += 64) {
        const uint32_t i = i0 + lane;
        bool samp = false;
        uint32_t qv = 0;
        if (i < cntw) {
            const uint32_t e = ent[srt[i]];
            const uint32_t lr = e & 63u, w0 = (e >> 6) & 0xFFu, n1 = (e >> 14) & 15u;
            const uint32_t p0 = rel[lr] + w0;
            uint4 o;
            o.x = sk_bases16(st, p0);
            o.y = sk_bases16(st, p0 + 16);
            o.z = (sk_bases16(st, p0 + 32) & 0x0FFFFFFFu) | n1 << 28;
            o.w = ((e >> 18) & ((1u << SK2_FBITS) - 1)) << 24 | ((rtile + lr) * M + w0);
            recs[base[e >> 26] + i] = o;
            samp = ((e >> 18) & smaskb) == 0;
            qv = p0 | n1 << 16;
        }
        const uint64_t sb = __builtin_amdgcn_ballot_w64(samp);
        if (samp) hq[nq + __builtin_amdgcn_mbcnt_hi((uint32_t)(sb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sb, 0u))] = qv;
        nq += (uint32_t)__popcll(sb);
        if (nq > (uint32_t)(SK2_HQ - 64)) hll_drain();
    }
    if (nq) hll_drain();
    wave_sync();
    if (lane < (uint32_t)C) wcnt[lane] = 0;
}

// Region of (c, g): records [(g * C + c) * cap, + cap) of recs, spill records at C * G * cap
// (SK2_ECAP_W of them: a flush stores at most that many; *overflow set, the call is redone); cnt[c * G + g] = records stored.
// elim (<= SK2_ECAP_W): the entries a wave may buffer (smaller only to test the overflow path).
// Entry (u32): lane | first window << 6 | (n - 1) << 14 | top SK2_BBITS of min_remix << 18.
// k_skpart_w: the partition for one compile-time window width W = k - m + 1 (the headline's k = 31: W = 17):
// a round is one block of W m-mers, their hashes and the previous block's suffix minima held
// in registers (van Herk / Gil-Werman: window rW + j = min(suffix_r[j], prefix_{r+1}[j - 1])),
// so no per-lane LDS ring; the buffer (no ring either) takes a whole round of entries.
//
// VAL (no k_prescan ran; M and the stage size come from the first read): the kernel checks
// what the prescan would have -- every read with windows is L = M + k - 1 bytes long, every
// byte of a read is A, C, G or T (decode(encode(byte)) == byte: one v_perm per 4 bytes), no
// tile outgrows the stage -- raises *vfail otherwise (the host then takes the prescan path),
// and adds the windows to *npos.
template <int NPF, int W, bool VAL>
__global__ void __launch_bounds__(PT_THREADS) k_skpart_w(const uint8_t *__restrict__ buf,
                                                         const uint64_t *__restrict__ off, uint64_t nreads, MinCfg mc,
                                                         uint32_t M, uint64_t gsize, uint32_t G, uint64_t cap,
                                                         uint32_t smask, uint4 *recs, unsigned int *cnt, uint8_t *hll,
                                                         unsigned long long *nrec, unsigned int *overflow,
                                                         unsigned int *vfail, unsigned long long *npos,
                                                         uint32_t g_lo, uint32_t elim) {
    constexpr int C = 1 << SK2_CBITS;
    constexpr int NREG = 1 << HLL_REG_BITS;
    constexpr int SW = NPF * 64 + 4;
    static_assert(SK2_FLUSH_AT >= 64, "the entry buffer holds a flush's worth");
    __shared__ uint32_t s_stage[PT_WAVES][SW];
    __shared__ uint32_t s_ent[PT_WAVES][SK2_ECAP_W];
    __shared__ uint16_t s_srt[PT_WAVES][SK2_ECAP_W];
    __shared__ uint32_t s_rel[PT_WAVES][64];
    __shared__ unsigned long long s_base[PT_WAVES][C];
    __shared__ unsigned int s_wcnt[PT_WAVES][C];
    __shared__ unsigned int s_cur[C];
    __shared__ unsigned int s_hll[NREG / 4];
    __shared__ uint32_t s_hq[PT_WAVES][SK2_HQ];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < NREG / 4; i += PT_THREADS) s_hll[i] = 0;
    if (threadIdx.x < C) s_cur[threadIdx.x] = 0;
    if (lane < C) s_wcnt[wid][lane] = 0;
    __syncthreads();
    const uint64_t g = blockIdx.x + (uint64_t)g_lo;  // (host input: launched per chunk of groups)
    const uint64_t g0 = min(g * gsize, nreads), g1 = min(g0 + gsize, nreads);
    const uint32_t ntile = (uint32_t)((g1 - g0 + 63) / 64);
    const int k = mc.k;
    constexpr uint32_t nmax = sk2_nmax(W + SK_M - 1);  // k = W + m - 1
    const uint64_t kmask = kmask64(k);
    uint4 pf[NPF];
    uint64_t nx_base = 0;
    uint32_t nx_s = 0, nx_e = 0, nx_n = 0, nx_lo = 0, nx_hi = 0, nx_n16 = 0;
    uint32_t nwin = 0;  // VAL: reads with windows (uniform)
    if (wid < ntile) EC_PT_ISSUE(wid);
    const unsigned long long gcap = g * C * cap, spill = (unsigned long long)C * G * cap;
    uint32_t *st = s_stage[wid];
    uint32_t *ent = s_ent[wid];
    for (uint32_t t = wid; t < ntile; t += PT_WAVES) {
        if (VAL) {
            // stage and check in one pass: x = the bytes' 2-bit codes (pack4's first step), a byte
            // is A, C, G or T iff decoding its code gives it back
            uint32_t diff = 0;
#pragma unroll
            for (int q = 0; q < NPF; q++) {
                const uint32_t wv[4] = {pf[q].x, pf[q].y, pf[q].z, pf[q].w};
                uint32_t packed = 0, d[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t x = ((wv[u] >> 1) ^ (wv[u] >> 2)) & 0x03030303u;
                    const uint32_t y = x | (x >> 6);
                    packed |= ((y | (y >> 12)) & 0xFFu) << (8 * u);
                    d[u] = __builtin_amdgcn_perm(0u, 0x54474341u, x) ^ wv[u];
                }
                st[q * 64 + lane] = packed;
                const uint32_t lo = 16 * (q * 64 + lane);  // the chunk's bytes relative to nx_base
                if (lo >= nx_lo && lo + 16 <= nx_hi) {
                    diff |= d[0] | d[1] | d[2] | d[3];
                } else if (lo < nx_hi && lo + 16 > nx_lo) {  // a chunk at the tile's ends: its read bytes only
                    // bytes [from, to) of the chunk are the tile's: a 16-bit byte mask, each dword's
                    // 4 bits widened to byte masks by one multiply
                    const uint32_t from = (uint32_t)min(max((int)nx_lo - (int)lo, 0), 16);
                    const uint32_t to = (uint32_t)min(max((int)nx_hi - (int)lo, 0), 16);
                    const uint32_t m16 = (0xFFFFu >> (16 - to)) & ~((1u << from) - 1u);
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t m4 = (m16 >> (4 * u)) & 15u;
                        const uint32_t keep = ((m4 * 0x00204081u) & 0x01010101u) * 0xFFu;
                        diff |= d[u] & keep;
                    }
                }
            }
            bool bad = nx_n16 > (uint32_t)NPF * 64 || diff != 0;  // a read longer than the stage, a byte
            if (lane < nx_n) {
                const uint32_t ln = nx_e - nx_s;
                bad |= ln >= (uint32_t)k && ln != M + (uint32_t)k - 1;
            }
            if (__any(bad) && lane == 0) atomicOr(vfail, 1u);
            nwin += (uint32_t)__popcll(__ballot(lane < nx_n && nx_e - nx_s >= (uint32_t)k));
        } else {
#pragma unroll
            for (int q = 0; q < NPF; q++) st[q * 64 + lane] = pack16(pf[q]);
        }
        const uint32_t tbase = (uint32_t)nx_base, s = nx_s;
        const uint32_t len = lane < nx_n ? nx_e - nx_s : 0u;
        const bool more = t + PT_WAVES < ntile;
        const bool has = len >= (uint32_t)k;  // then len - k + 1 == M
        const uint32_t rel = has ? s - tbase : 0u;
        s_rel[wid][lane] = rel;
        wave_sync();
        constexpr int m = SK_M;
        constexpr uint32_t MMASK = (1u << (2 * SK_M)) - 1;
        uint32_t mf = 0, mr = 0;
        auto push_base = [&](uint32_t b) {
            mf = ((mf << 2) | b) & MMASK;
            mr = (mr >> 2) | ((3u - b) << (2 * SK_M - 2));
        };
        // block 0 = m-mers 0 .. W - 1 (bases 0 .. k - 1): its suffix minima
        uint32_t S[W];
        {
            const uint32_t x0 = sk_bases16(st, rel), x1 = sk_bases16(st, rel + 16);
#pragma unroll
            for (int tb = 0; tb < m - 1; tb++) push_base(tb < 16 ? (x0 >> (2 * tb)) & 3u : (x1 >> (2 * (tb - 16))) & 3u);
#pragma unroll
            for (int j = 0; j < W; j++) {
                const int tb = m - 1 + j;
                push_base(tb < 16 ? (x0 >> (2 * tb)) & 3u : (x1 >> (2 * (tb - 16))) & 3u);
                S[j] = mmer_hash(mf < mr ? mf : mr);
            }
#pragma unroll
            for (int j = W - 2; j >= 0; j--) S[j] = min(S[j], S[j + 1]);
        }
        const uint32_t nrounds = __any(has) ? (M + W - 1) / W : 0u;
        // the open run of a lane: windows [rs, w) of minimizer runv.  runv starts as window 0's
        // value, so window 0 never closes a run; a lane without a read never closes one (has).
        // The run start is kept as its entry term rsx = -16320 rs (below): the close test
        // rs == end - nmax compares it with a uniform constant and the entry needs no multiply
        uint32_t runv = S[0], rsx = 0, cntw = 0;  // cntw: the wave's buffered entries (uniform)
        const uint64_t hasm = __builtin_amdgcn_ballot_w64(has);
        const uint32_t rtile = 64 * t;            // the tile's first read relative to g0
        // entry of the run [rs, end) closing at window end: lane | rs << 6 | (n - 1) << 14 |
        // bucket bits << 18 with n = end - rs (fields disjoint, so a sum: (end - 1) << 14 -
        // 16320 rs), the bucket bits the top 14 of min_remix(runv) = its low 14 (the shift drops
        // the rest)
        auto entry = [&](uint32_t end) { return (runv << 18) + lane + (((end - 1u) << 14) + rsx); };
        auto rs_term = [](uint32_t w) { return (uint32_t)((int)w * -16320); };
        for (uint32_t round = 0; round < nrounds; round++) {
            const uint32_t w0 = round * W;  // first window of the round
            // m-mer (round + 1) W + j covers bases q + j .. q + j + m - 1: a0, a1 = bases q .. q + 31
            // (W + m - 1 <= 32).  Its forward code rolls in base q + m - 1 + j; its reverse
            // complement's code is the complement of the m bases read little-endian (base i at
            // bits 2i), one alignbit -- no second rolling register
            const uint32_t q = rel + w0 + W;
            const uint32_t a0 = sk_bases16(st, q), a1 = sk_bases16(st, q + 16);
            const uint32_t rw0 = rs_term(w0);  // (uniform: window w0 + j's term is rw0 + rs_term(j))
            uint32_t H[W];
            uint32_t P = 0xFFFFFFFFu;  // prefix minimum of the next block so far
            // one window: its minimizer v, the next block's hash j, and the run bookkeeping.  A run
            // closes when the minimizer changes or it holds nmax windows: the closing lanes append
            // their entries (ballot rank), the others only move rs
            auto window = [&](int j) {
                const uint32_t v = min(S[j], P);  // window w0 + j
                const int tb = m - 1 + j;  // the rolled-in base, relative to q
                const uint32_t b = tb < 16 ? (a0 >> (2 * tb)) & 3u : (a1 >> (2 * (tb - 16))) & 3u;
                mf = (mf << 2) | b;  // (bits past the m-mer's 2m are dropped where it is used)
                const uint32_t fw = mf & MMASK;
                const uint32_t le = j == 0 ? a0 : j < 16 ? __builtin_amdgcn_alignbit(a1, a0, 2 * j) : a1 >> (2 * (j - 16));
                const uint32_t rc = ~le & MMASK;
                H[j] = mmer_hash(fw < rc ? fw : rc);
                P = min(P, H[j]);
                const uint32_t end = w0 + j;  // uniform
                // (the mask from the compares' own ballots: a ballot of the combined bool was
                // materialised through a VGPR)
                const bool c1 = v != runv, c2 = rsx == rw0 + (uint32_t)((j - (int)nmax) * -16320);
                const bool close = has & (c1 | c2);
                const uint64_t bal = (__builtin_amdgcn_ballot_w64(c1) | __builtin_amdgcn_ballot_w64(c2)) & hasm;
                if (close) {
                    const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    ent[min(cntw, elim - 64) + rk] = entry(end);  // (a uniform clamp: in bounds; past it, *overflow)
                    rsx = rw0 + (uint32_t)(j * -16320);
                }
                cntw += (uint32_t)__popcll(bal);
                runv = v;
            };
            if (w0 + W <= M) {  // a whole round: no bound checks
#pragma unroll
                for (int j = 0; j < W; j++) window(j);
            } else {
#pragma unroll
                for (int j = 0; j < W; j++) {
                    if (w0 + j >= M) break;  // uniform
                    window(j);
                }
            }
            // the next round's suffix minima (the block's unused tail at the read's end is never read)
#pragma unroll
            for (int j = 0; j < W; j++) S[j] = H[j];
#pragma unroll
            for (int j = W - 2; j >= 0; j--) S[j] = min(S[j], S[j + 1]);
            if (cntw > elim - 64) {  // entries were stored over others: the call is redone
                if (lane == 0) atomicOr(overflow, 1u);
                cntw = elim - 64;
            }
            // flush: the buffer may not take another round
            if (round + 1 < nrounds && cntw > elim - 64 - 640) {
                skpart_flush<C>(cntw, ent, s_srt[wid], s_wcnt[wid], s_cur, s_base[wid], s_rel[wid], st, lane, gcap,
                                cap, spill, M, rtile, recs, overflow, s_hll, s_hq[wid], smask ? 0xFFu : 0u, k,
                                kmask);
                cntw = 0;
            }
        }
        // the next tile's loads go in flight here, past the rounds, on every path (the last tile
        // reloads itself): the prefetch registers are then dead while the windows run -- issued
        // inside the last round, they stayed live through every round (28 VGPRs at NPF = 7)
        EC_PT_ISSUE(more ? t + PT_WAVES : t);
        if (nrounds) {  // the reads' final runs (windows [rs, M)), then the stage's last flush
            const uint64_t bal = hasm;
            if (has) {
                const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                ent[cntw + rk] = entry(M);  // (cntw <= elim - 64 here)
            }
            cntw += (uint32_t)__popcll(bal);
            skpart_flush<C>(cntw, ent, s_srt[wid], s_wcnt[wid], s_cur, s_base[wid], s_rel[wid], st, lane, gcap,
                            cap, spill, M, rtile, recs, overflow, s_hll, s_hq[wid], smask ? 0xFFu : 0u, k, kmask);
        }
    }
    __shared__ unsigned int s_nwin[PT_WAVES];
    if (VAL && lane == 0) s_nwin[wid] = nwin;
    __syncthreads();
    if (threadIdx.x < C) cnt[(uint64_t)threadIdx.x * G + g] = (unsigned int)min((uint64_t)s_cur[threadIdx.x], cap);
    if (threadIdx.x == 0) {  // records (and VAL: windows) of the group, one atomic each per workgroup
        unsigned long long tot = 0;
        for (int c = 0; c < C; c++) tot += s_cur[c];
        if (tot) atomicAdd(nrec, tot);
        if (VAL) {
            unsigned long long wn = 0;
            for (int q = 0; q < PT_WAVES; q++) wn += s_nwin[q];
            if (wn) atomicAdd(npos, wn * M);
        }
    }
    unsigned int *hw = reinterpret_cast<unsigned int *>(hll + g * NREG);
    for (int i = threadIdx.x; i < NREG / 4; i += PT_THREADS) hw[i] = s_hll[i];
}

// ---- refine: (group, coarse) runs -> fixed-capacity final buckets ------------------------------
// As k_refine2: workgroup (c, y) reads the runs of groups [G y / RS, G (y + 1) / RS) of coarse
// bucket c, sorts SK2_TILE-record tiles by final bucket in LDS and appends each final bucket's
// run at a cursor reserved by one global atomic: final bucket b holds [b fcap, b fcap + fcur[b]).
__global__ void __launch_bounds__(BUCKET_THREADS) k_skrefine(const uint4 *recs, const unsigned int *cnt, uint32_t G,
                                                             uint64_t cap, int bbits, uint4 *out, uint64_t fcap,
                                                             unsigned long long *fcur, unsigned int *overflow,
                                                             uint32_t M, uint64_t gsize, uint64_t read_base) {
    constexpr int TILE = SK2_TILE;
    constexpr int PER = TILE / BUCKET_THREADS;
    constexpr uint64_t C = 1 << SK2_CBITS;
    __shared__ uint4 tile[TILE];
    __shared__ uint8_t tj[TILE];
    __shared__ unsigned long long base[REFINE_FANOUT];
    __shared__ unsigned int tcnt[REFINE_FANOUT], tbeg[REFINE_FANOUT], wsum[BUCKET_THREADS / 64];
    __shared__ unsigned int lst[RF_MAX_RUNS + 1];
    const int fb = bbits - SK2_CBITS;  // final bits below the coarse bits
    const int F = 1 << fb;
    const uint64_t c = blockIdx.x;
    const uint32_t ga = (uint32_t)((uint64_t)G * blockIdx.y / gridDim.y),
                   gb = (uint32_t)((uint64_t)G * (blockIdx.y + 1) / gridDim.y);
    const uint32_t nr = gb - ga;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    {
        const uint32_t i0 = 2 * threadIdx.x;
        const unsigned int a = i0 < nr ? cnt[c * G + ga + i0] : 0u, b = i0 + 1 < nr ? cnt[c * G + ga + i0 + 1] : 0u;
        unsigned int incl = a + b;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        unsigned int before = 0;
        for (int q = 0; q < wid; q++) before += wsum[q];
        const unsigned int ex = before + incl - (a + b);
        if (i0 <= nr) lst[i0] = ex;
        if (i0 + 1 <= nr) lst[i0 + 1] = ex + a;
        __syncthreads();
    }
    const uint64_t N = lst[nr];
    uint32_t j0 = 0;
    for (uint64_t t0 = 0; t0 < N; t0 += TILE) {
        while (j0 + 1 < nr && lst[j0 + 1] <= t0) j0++;
        const unsigned int n = (unsigned int)min((uint64_t)TILE, N - t0);
        if (threadIdx.x < REFINE_FANOUT) tcnt[threadIdx.x] = 0;
        __syncthreads();
        // (plain u32 arrays: an array of uint4 was kept in memory, not registers)
        unsigned int rx[PER], ry[PER], rz[PER], rw[PER], lr[PER], jj[PER], rk[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                const uint64_t l = t0 + i;
                uint32_t jr = j0;
                while (lst[jr + 1] <= l) jr++;
                const uint4 v = recs[((ga + jr) * C + c) * cap + (l - lst[jr])];
                rx[q] = v.x, ry[q] = v.y, rz[q] = v.z, rw[q] = v.w;
                lr[q] = jr;
            }
        }
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                jj[q] = fb ? (rw[q] >> 24) >> (SK2_FBITS - fb) : 0u;
                rw[q] = (uint32_t)((read_base + (uint64_t)(ga + lr[q]) * gsize) * M) + (rw[q] & 0xFFFFFFu);
                rk[q] = atomicAdd(&tcnt[jj[q]], 1u);
            }
        }
        __syncthreads();
        unsigned long long mybase = 0;
        unsigned int myv = 0;
        if (threadIdx.x < REFINE_FANOUT) {
            const unsigned int v = (int)threadIdx.x < F ? tcnt[threadIdx.x] : 0u;
            unsigned int incl = v;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int u = __shfl_up(incl, o);
                if (lane >= o) incl += u;
            }
            tbeg[threadIdx.x] = incl - v;
            if (lane == 63) wsum[wid] = incl;
            myv = v;
            if (v) mybase = atomicAdd(&fcur[c * F + threadIdx.x], (unsigned long long)v);
        }
        __syncthreads();
        if (threadIdx.x >= 64 && threadIdx.x < REFINE_FANOUT) {
            unsigned int add = 0;
            for (int q = 0; q < (int)(threadIdx.x >> 6); q++) add += wsum[q];
            tbeg[threadIdx.x] += add;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = threadIdx.x + q * BUCKET_THREADS;
            if (i < n) {
                const unsigned int p = tbeg[jj[q]] + rk[q];
                tile[p] = make_uint4(rx[q], ry[q], rz[q], rw[q]);
                tj[p] = (uint8_t)jj[q];
            }
        }
        if (threadIdx.x < REFINE_FANOUT) {
            if (mybase + myv > fcap) atomicOr(overflow, 1u);
            base[threadIdx.x] = (c * F + threadIdx.x) * fcap + mybase;
            tcnt[threadIdx.x] = mybase < fcap ? (unsigned int)min<unsigned long long>(fcap - mybase, 0xFFFFFFFFull) : 0u;
        }
        __syncthreads();
        for (unsigned int i = threadIdx.x; i < n; i += BUCKET_THREADS) {
            const unsigned int j = tj[i];
            const unsigned int q = i - tbeg[j];
            if (q < tcnt[j]) out[base[j] + q] = tile[i];
        }
        __syncthreads();
    }
}

// ---- bucket: super-k-mers -> LDS table
// The bucket table of k_skbucket: count_part.h's LTab with 32-bit first events
// e = read * 2M + l (ordered as (read, l); phase_count_sk2 checks (read_base + reads) * 2M <
// 2^32) and no id words -- 40 KiB for 2048 slots instead of 64, its event read 8 bytes.
template <int SLOTS>
struct LTabE {
    unsigned long long key[SLOTS];
    uint2 ev[SLOTS];
    unsigned int count[SLOTS];
};
struct EvExpand {  // e -> (read << 32) | l for the dense arrays
    unsigned int m2;  // 2M
    __device__ inline unsigned long long one(unsigned int e) const {
        return ((unsigned long long)(e / m2) << 32) | (e % m2);
    }
    template <typename Tab>
    __device__ inline ulonglong2 operator()(const Tab &tab, int i) const {
        return make_ulonglong2(one(tab.ev[i].x), one(tab.ev[i].y));
    }
};


// ---- bucket with the bucket's duplicate super-k-mers merged first (the default) -----------------
// At ~150-fold coverage a bucket's records are mostly the same few super-k-mers read again and
// again (each interior super-k-mer of the genome appears in ~130 reads, in two orientations).  The
// records first go through an LDS table keyed by their CANONICAL content -- the L = n + k - 1
// bases masked to L (the partition copies bases past the run too) or their reverse complement,
// whichever is smaller, plus n -- keeping per distinct record its multiplicity and two event
// minima: with A = read 2M + first window and B = read 2M + 2M - 1 - first window, window o's
// k-mer string was inserted by build() at A + o and its twin at B - o (count_part.h events); a
// record taken in reverse complement has A' = B - n + 1, B' = A + n - 1 (window o' of the flip is
// the twin of window n - 1 - o).  Identical canonical records have identical window strings, so
// min over copies of (A + o) = min A + o: the distinct records insert their windows once, with
// add = multiplicity, and every key's count and first events equal the per-record inserts'.
// The record table takes up to RS / 2 distinct records; a record that finds no entry once it is
// that full is rolled out on its own (any split of the copies between entries is exact).
// Probing claims a slot by CAS on a tag word (20 hash bits | PEND), stores the key and publishes
// it by clearing PEND (release); a prober compares keys only behind a published tag (acquire), so
// no barrier is needed -- a record that meets a pending slot of its own key just takes another
// entry.  Each thread takes RB records per round: their loads, canonical forms and probe chains
// overlap (one record per thread was bound by the latency of its dependent LDS round trips).
__device__ inline uint32_t rev2_32b(uint32_t v) {  // superkmer.h rev2_32 with one v_bfrev_b32
    v = __builtin_bitreverse32(v);
    return ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
}

template <int SLOTS, int RS, int RB, bool EVEN_K>
__global__ void __launch_bounds__(BUCKET_THREADS) k_skbucket(const uint4 *recs, const unsigned long long *bbeg,
                                                             const unsigned long long *bend, int k, uint32_t M,
                                                             double inv_m, long long limit, unsigned long long *dkey,
                                                             unsigned int *dcnt, unsigned long long *dfc,
                                                             unsigned long long *dft, SubSlot *sub,
                                                             unsigned int *nsolid, unsigned long long *ndistinct,
                                                             unsigned int *overflow, unsigned long long *dbg) {
    constexpr int SBITS = SLOTS == 2048 ? 11 : 12;
    constexpr uint32_t PEND = 0x800u;  // tag word: the claimer has not yet stored the key
    // entries claimed at most: half the slots, and low enough that the claims a block can have in
    // flight past the check (one per record being probed) still leave a free slot
    constexpr unsigned int CLAIM_MAX = RS / 2 < RS - 1 - RB * BUCKET_THREADS ? RS / 2 : RS - 1 - RB * BUCKET_THREADS;
    static_assert(RS > RB * BUCKET_THREADS + 1, "record table too small for the records in flight");
    __shared__ LTabE<SLOTS> tab;
    __shared__ unsigned int s_over[2];
    __shared__ uint32_t r_tag[RS], r_x[RS], r_y[RS], r_z[RS], r_mult[RS], r_a[RS], r_b[RS];
    __shared__ uint16_t s_ord[RS];
    __shared__ unsigned int s_nent, s_ncnt[SK2_NMAX + 1];
    const unsigned int b = blockIdx.x, tid = threadIdx.x;
    for (int i = tid; i < SLOTS; i += BUCKET_THREADS) {
        tab.key[i] = EMPTY_KEY;
        tab.count[i] = 0;
        tab.ev[i] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    }
    for (int i = tid; i < RS; i += BUCKET_THREADS) {
        r_tag[i] = 0;
        r_mult[i] = 0;
        r_a[i] = r_b[i] = 0xFFFFFFFFu;
    }
    if (tid <= SK2_NMAX) s_ncnt[tid] = 0;
    if (tid == 0) s_over[0] = s_over[1] = 0, s_nent = 0;
    // EULERHIP_SK2_STATS: per-phase wall clock (100 MHz) summed over the blocks, thread 0's view
    unsigned long long t_last = 0;
    auto phase = [&](int i) {
        if (dbg && tid == 0) {
            const unsigned long long t = wall_clock64();
            if (i) atomicAdd(&dbg[2 + i], t - t_last);
            t_last = t;
        }
    };
    phase(0);
    __syncthreads();
    const uint64_t r0 = bbeg[b], r1 = bend[b];
    const uint64_t kmask = kmask64(k);
    const int sh = 2 * (k - 1), fsh = 64 - 2 * k;
    const unsigned int m2 = 2 * M - 1, M2 = 2 * M;

    unsigned long long n_rolled = 0;  // (EULERHIP_SK2_STATS; no global atomics in the loops: they
                                      // would hold the record loads' counter at vmcnt(0))
    // the n windows of a (canonical) record into the k-mer table: window o's string was inserted
    // at ea + o, its twin at eb - o, mult times each
    auto roll_out = [&](uint32_t x0, uint32_t x1, uint32_t x2, unsigned int mult, unsigned int ea, unsigned int eb) {
        const unsigned int n = (x2 >> 28) + 1;
        if (dbg) n_rolled += n;
        auto events = [&](uint64_t fwd, uint64_t rc, unsigned int o, unsigned int &eC, unsigned int &eT,
                          unsigned int &add) {
            const bool tw = fwd > rc;
            const unsigned int ef = ea + o, et = eb - o;
            add = mult;
            eC = tw ? et : ef;
            eT = tw ? ef : et;
            if (EVEN_K && fwd == rc) {  // even-k palindrome: both inserts at its first event
                add = 2 * mult;
                eC = eT = min(ef, et);
            }
            return tw ? rc : fwd;
        };
        const unsigned int h = (n + 1) >> 1;  // two windows per step (o and o + h)
        auto at = [&](unsigned int o, uint64_t &fw, uint64_t &rv) {  // window o straight out of the bases
            const uint32_t lo = __builtin_amdgcn_alignbit(x1, x0, 2 * o), hi = __builtin_amdgcn_alignbit(x2, x1, 2 * o);
            const uint64_t P = (uint64_t)lo | (uint64_t)hi << 32;
            rv = ~P & kmask;
            fw = rev2_64(P) >> fsh;
        };
        auto roll = [&](unsigned int o, uint64_t &fw, uint64_t &rv) {  // to window o from o - 1
            const unsigned int tb = o + (unsigned int)k - 1;
            const uint32_t wd = tb < 32 ? x1 : x2;
            const uint32_t bb = (wd >> (2 * (tb & 15))) & 3u;
            fw = ((fw << 2) | bb) & kmask;
            rv = (rv >> 2) | ((uint64_t)(3u - bb) << sh);
        };
        uint64_t fA, rA, fB, rB;
        at(0, fA, rA);
        at(h, fB, rB);
        for (unsigned int i = 0; i < h; i++) {
            const unsigned int oB = i + h;
            const bool bB = oB < n;
            if (i) {
                roll(i, fA, rA);
                roll(oB, fB, rB);
            }
            unsigned int eCA, eTA, eCB, eTB, addA, addB;
            const uint64_t cA = events(fA, rA, i, eCA, eTA, addA);
            const uint64_t cB = events(fB, rB, oB, eCB, eTB, addB);
            unsigned int sA = (sk_slot(cA) >> (32 - SBITS)) & (SLOTS - 1), sB = (sk_slot(cB) >> (32 - SBITS)) & (SLOTS - 1);
            const unsigned long long kA = tab.key[sA], kB = tab.key[sB];
            lds_locate2<SLOTS>(tab, s_over, cA, sA, kA, cB, sB, bB ? kB : cB);
            atomicAdd(&tab.count[sA], addA);
            if (bB) atomicAdd(&tab.count[sB], addB);
            const uint2 vA = tab.ev[sA], vB = tab.ev[sB];
            if (eCA < vA.x) atomicMin(&tab.ev[sA].x, eCA);
            if (eTA < vA.y) atomicMin(&tab.ev[sA].y, eTA);
            if (bB && eCB < vB.x) atomicMin(&tab.ev[sB].x, eCB);
            if (bB && eTB < vB.y) atomicMin(&tab.ev[sB].y, eTB);
        }
    };

    // ---- records -> record table (no barrier: a slot's key is published by clearing PEND) ----
    // RB records per thread and round, their loads, canonical forms and probe chains in flight
    // together (one record per thread waited on its global load and on a chain of dependent
    // LDS round trips: latency-bound)
    constexpr unsigned int ROUND = RB * BUCKET_THREADS;
    phase(1);  // [3] init
    // records PD rounds ahead in flight per thread (one round ahead left the loads' latency
    // exposed once the probes were cheap: ~16 KiB in flight per CU); the round loop is unrolled
    // PD times so each slot is consumed and reloaded in place (no register moves that would wait)
    constexpr int PD = SK2_PD;
    uint4 nx[PD][RB];
#pragma unroll
    for (int d = 0; d < PD; d++)
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const uint64_t ri = r0 + tid + (uint64_t)j * BUCKET_THREADS + (uint64_t)d * ROUND;
            nx[d][j] = recs[r1 > r0 ? min(ri, r1 - 1) : r0];  // (an empty bucket reads its own start)
        }
    // EULERHIP_SK2_STATS: per-wave shader-clock split of the records phase (dbg[8..13])
    unsigned long long c_canon = 0, c_probe = 0, c_post = 0, n_iter = 0, n_rounds = 0, c_t = 0;
    auto tick = [&](unsigned long long &acc) {
        if (dbg) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc += t - c_t;
            c_t = t;
        }
    };
    if (dbg) c_t = __builtin_amdgcn_s_memtime();
    auto record_round = [&](uint4 (&nxd)[RB], uint64_t c0) {
        if (dbg) n_rounds++;
        uint32_t K0[RB], K1[RB], K2[RB], EA[RB], EB[RB], TG[RB], SL[RB];
        int ST[RB];  // 0 searching, 1 found / claimed, 2 table full (rolled out on its own)
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const uint64_t ri = c0 + tid + (uint64_t)j * BUCKET_THREADS;
            const bool valid = ri < r1;
            const uint4 x = nxd[j];
            // the records PD rounds on; unconditional (clamped; the value past the end is not
            // used), so the loads stay in order in flight and the wait before use is vmcnt(PD - 1)
            nxd[j] = recs[min(ri + PD * ROUND, r1 - 1)];
            // canonical content of the record (branch-free: selects, no divergent paths)
            const unsigned int n = (x.z >> 28) + 1, L2 = 2 * (n + (unsigned int)k - 1);  // 2L in [2k, 92]
            const uint32_t m1 = L2 >= 64 ? 0xFFFFFFFFu : (1u << ((L2 - 32) & 31)) - 1u;  // bits of word 1
            const uint32_t mw2 = L2 > 64 ? (1u << ((L2 - 64) & 31)) - 1u : 0u;           // bits of word 2
            const uint32_t x0 = x.x, x1 = x.y & m1, x2 = x.z & mw2;
            // reverse complement of the L bases: rev2 of the 96-bit string (base i -> 47 - i), then
            // down by 96 - 2L bits (4 .. 54), complemented
            const uint32_t y0 = rev2_32b(x2), y1 = rev2_32b(x1), y2 = rev2_32b(x0);
            const unsigned int sft = 96 - L2, s5 = sft & 31;
            const bool lo = sft < 32;
            const uint32_t a0 = __builtin_amdgcn_alignbit(y1, y0, s5), a1 = __builtin_amdgcn_alignbit(y2, y1, s5),
                           a2 = y2 >> s5;
            const uint32_t q0 = ~(lo ? a0 : a1), q1 = ~(lo ? a1 : a2) & m1, q2 = lo ? ~a2 & mw2 : 0u;
            const bool flip = q2 != x2 ? q2 < x2 : q1 != x1 ? q1 < x1 : q0 < x0;
            // events of window 0: A = read 2M + first window, B = read 2M + 2M - 1 - first window
            const unsigned int p = x.w;
            const unsigned int rd0 = (unsigned int)((double)p * inv_m);  // p / M, corrected below
            int rm = (int)(p - rd0 * M);
            unsigned int rd = rd0;
            if (rm < 0) rd--, rm += (int)M;
            else if (rm >= (int)M) rd++, rm -= (int)M;
            const unsigned int A = rd * M2 + (unsigned int)rm, B = rd * M2 + m2 - (unsigned int)rm;
            K0[j] = flip ? q0 : x0, K1[j] = flip ? q1 : x1, K2[j] = (flip ? q2 : x2) | (n - 1) << 28;
            EA[j] = flip ? B - n + 1 : A, EB[j] = flip ? A + n - 1 : B;
            // content hash -> first slot, tag
            uint32_t hh = K0[j] * 0x9E3779B1u;
            hh = (hh ^ (hh >> 15) ^ K1[j]) * 0x85EBCA77u;
            hh = (hh ^ (hh >> 13) ^ K2[j]) * 0xC2B2AE3Du;
            hh ^= hh >> 16;
            TG[j] = (hh | 0x1000u) & 0xFFFFF000u;
            SL[j] = __umulhi(hh * 0x27D4EB2Fu, (unsigned int)RS);
            ST[j] = valid ? 0 : 1;
        }
        auto searching = [&]() {
            bool a = false;
#pragma unroll
            for (int j = 0; j < RB; j++) a |= ST[j] == 0;
            return a;
        };
        // a step reads every chain's tag and key words (in program order: a published tag read
        // first implies the key words read after it are the stored key -- DS operations of a wave
        // complete in order), compares branch-free, and only the rare empty slot takes the claim
        // path; a chain that is done re-reads its slot harmlessly
        // (relaxed atomic loads stay ds_read_b32 with one wait for all four; volatile pointers
        // had lost the LDS address space: flat loads with a full wait after each, 4x slower)
        auto ld = [](uint32_t *a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
        tick(c_canon);
#pragma unroll 1
        while (__any(searching())) {
            if (dbg) n_iter++;
            uint32_t T[RB], X[RB], Y[RB], Z[RB];
#pragma unroll
            for (int j = 0; j < RB; j++) T[j] = ld(&r_tag[SL[j]]);
            asm volatile("" ::: "memory");  // the key words are read after the tag (issue order)
#pragma unroll
            for (int j = 0; j < RB; j++) X[j] = ld(&r_x[SL[j]]), Y[j] = ld(&r_y[SL[j]]), Z[j] = ld(&r_z[SL[j]]);
            bool claim = false;
#pragma unroll
            for (int j = 0; j < RB; j++) {
                const bool hit = T[j] == TG[j] && X[j] == K0[j] && Y[j] == K1[j] && Z[j] == K2[j];
                const bool go = ST[j] == 0;
                ST[j] = go && hit ? 1 : ST[j];
                claim |= go && !hit && T[j] == 0;
                // a published tag of another key, or a pending one of other tag bits: the next slot;
                // a pending slot of this tag is read again (its claimer publishes within a few
                // instructions), so concurrent copies of a new record share one entry
                if (go && !hit && T[j] != 0 && T[j] != (TG[j] | PEND))
                    SL[j] = SL[j] + 1 == (unsigned int)RS ? 0u : SL[j] + 1;
            }
            if (claim) {
#pragma unroll
                for (int j = 0; j < RB; j++) {
                    if (ST[j] != 0 || T[j] != 0) continue;
                    const unsigned int slot = SL[j];
                    // claims stop at CLAIM_MAX entries (a plain read: at most a block's worth of
                    // claims in flight overshoot it, so free slots always remain and a miss meets
                    // one within a few probes -- linear probing near full scans the table)
                    if (ld(&s_nent) >= CLAIM_MAX) {
                        ST[j] = 2;
                    } else if (atomicCAS(&r_tag[slot], 0u, TG[j] | PEND) == 0) {  // store the key, publish
                        r_x[slot] = K0[j], r_y[slot] = K1[j], r_z[slot] = K2[j];
                        __hip_atomic_store(&r_tag[slot], TG[j], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        atomicAdd(&s_nent, 1u);
                        ST[j] = 1;
                    }  // (lost the race: the slot is read again next step)
                }
            }
        }
        tick(c_probe);
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const bool valid = c0 + tid + (uint64_t)j * BUCKET_THREADS < r1;
            if (valid && ST[j] == 1) {
                const unsigned int slot = SL[j];
                atomicAdd(&r_mult[slot], 1u);
                if (EA[j] < r_a[slot]) atomicMin(&r_a[slot], EA[j]);
                if (EB[j] < r_b[slot]) atomicMin(&r_b[slot], EB[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < RB; j++)
            if (ST[j] == 2) roll_out(K0[j], K1[j], K2[j], 1u, EA[j], EB[j]);
        tick(c_post);
    };
    for (uint64_t c0 = r0; c0 < r1; c0 += PD * ROUND) {
#pragma unroll
        for (int d = 0; d < PD; d++) {
            if (c0 + (uint64_t)d * ROUND >= r1) break;  // uniform
            record_round(nx[d], c0 + (uint64_t)d * ROUND);
        }
    }
    unsigned long long c_bar = 0;
    __syncthreads();
    tick(c_bar);
    if (dbg && (tid & 63) == 0) {
        atomicAdd(&dbg[8], c_canon), atomicAdd(&dbg[9], c_probe), atomicAdd(&dbg[10], c_post);
        atomicAdd(&dbg[11], n_iter), atomicAdd(&dbg[12], c_bar), atomicAdd(&dbg[13], n_rounds);
    }
    phase(2);  // [4] records (thread 0 + the barrier)
    // ---- the distinct records into the k-mer table, by window count (most first) -------------
    {
        constexpr int PER = (RS + BUCKET_THREADS - 1) / BUCKET_THREADS;
        unsigned int sl[PER], rk[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const unsigned int i = tid + q * BUCKET_THREADS;
            sl[q] = SK2_NMAX;
            if (i < (unsigned)RS && r_tag[i]) {
                sl[q] = SK2_NMAX - 1 - (r_z[i] >> 28);
                rk[q] = atomicAdd(&s_ncnt[sl[q]], 1u);
            }
        }
        __syncthreads();
        if (tid == 0) {
            unsigned int a = 0;
            for (int q = 0; q < SK2_NMAX; q++) {
                const unsigned int v = s_ncnt[q];
                s_ncnt[q] = a;
                a += v;
            }
            s_ncnt[SK2_NMAX] = a;
            if (dbg) atomicAdd(&dbg[0], (unsigned long long)a), atomicAdd(&dbg[1], 1ull);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; q++)
            if (sl[q] < SK2_NMAX) s_ord[s_ncnt[sl[q]] + rk[q]] = (uint16_t)(tid + q * BUCKET_THREADS);
        __syncthreads();
        const unsigned int ne = s_ncnt[SK2_NMAX];
        phase(3);  // [5] sort
        if (dbg) c_t = __builtin_amdgcn_s_memtime();
        unsigned long long c_roll = 0, c_bar2 = 0;
        for (unsigned int t = tid; t < ne; t += BUCKET_THREADS) {
            const unsigned int e = s_ord[t];
            roll_out(r_x[e], r_y[e], r_z[e], r_mult[e], r_a[e], r_b[e]);
        }
        tick(c_roll);
        __syncthreads();
        tick(c_bar2);
        if (dbg && (tid & 63) == 0) atomicAdd(&dbg[14], c_roll), atomicAdd(&dbg[15], c_bar2);
        if (dbg) atomicAdd(&dbg[2], n_rolled);
    }
    phase(4);  // [6] roll-out
    lds_table_finish<SLOTS, false, KeyId>(tab, s_over, b, limit, dkey, dcnt, dfc, dft, sub, nsolid, ndistinct,
                                          overflow, KeyId(), EvExpand{2 * M});
    phase(5);  // [7] finish
}


// ---- k_skbucket3: small buckets, several workgroups per CU ------------------------------------
// k_skbucket's 133 KiB of LDS (the 3072-entry record table beside the 2048-slot k-mer table) held
// one workgroup per CU: its barriers, the init and the per-bucket tail were exposed.  Here a
// bucket is half as large (2^14 buckets, ~280 keys: a 1024-slot k-mer table) and the two tables
// share one region: the record table in the records phase, then the k-mer table beside the
// distinct records compacted (sorted by window count) out of it.  NT = 512 threads and ~50 KiB
// of LDS: three workgroups per CU.  Records the record table cannot take (past CLAIM_MAX
// entries) wait in a small overflow list and are rolled out after the distinct ones; a full
// list raises *overflow (the call is redone on another path).
template <int SLOTS, int RS, int NT>
struct SkB3Lds {
    static constexpr int NC = RS / 2;  // compact records (CLAIM_MAX <= RS / 2)
    struct Rec {
        uint32_t tag[RS], x[RS], y[RS], z[RS], mult[RS], a[RS], b[RS];
    };
    struct Roll {
        LTabE<SLOTS> tab;
        uint32_t x[NC], y[NC], z[NC], mult[NC], a[NC], b[NC];
    };
    union {
        Rec r;
        Roll k;
    };
};

template <int SLOTS, int RS, int NT, bool EVEN_K>
__global__ void __launch_bounds__(NT) k_skbucket3(const uint4 *recs, const unsigned long long *bbeg,
                                                  const unsigned long long *bend, int k, uint32_t M, double inv_m,
                                                  long long limit, unsigned long long *dkey, unsigned int *dcnt,
                                                  unsigned long long *dfc, unsigned long long *dft, SubSlot *sub,
                                                  unsigned int *nsolid, unsigned long long *ndistinct,
                                                  unsigned int *overflow, unsigned long long *dbg,
                                                  unsigned int claim_cap, unsigned int *bmark = nullptr) {
    constexpr int SBITS = __builtin_ctz(SLOTS);
    constexpr uint32_t PEND = 0x800u;
    constexpr unsigned int CLAIM_MAX = RS / 2 < RS - 1 - NT ? RS / 2 : RS - 1 - NT;
    static_assert(RS > NT + 1, "record table too small for the records in flight");
    static_assert(sizeof(typename SkB3Lds<SLOTS, RS, NT>::Roll) <= sizeof(typename SkB3Lds<SLOTS, RS, NT>::Rec),
                  "the k-mer table and the compact records fit the record table's space");
    constexpr int OV = 256;  // overflow list
    __shared__ SkB3Lds<SLOTS, RS, NT> L;
    __shared__ uint32_t o_x[OV], o_y[OV], o_z[OV], o_a[OV], o_b[OV];
    __shared__ unsigned int s_over[2];
    __shared__ unsigned int s_nent, s_nov, s_ncnt[SK2_NMAX + 1];
    auto &R = L.r;
    auto &tab = L.k.tab;
    const unsigned int b = blockIdx.x, tid = threadIdx.x;
    for (int i = tid; i < RS; i += NT) {
        R.tag[i] = 0;
        R.mult[i] = 0;
        R.a[i] = R.b[i] = 0xFFFFFFFFu;
    }
    if (tid <= SK2_NMAX) s_ncnt[tid] = 0;
    if (tid == 0) s_over[0] = s_over[1] = 0, s_nent = 0, s_nov = 0;
    __syncthreads();
    const uint64_t r0 = bbeg[b], r1 = bend[b];
    const uint64_t kmask = kmask64(k);
    const int sh = 2 * (k - 1), fsh = 64 - 2 * k;
    const unsigned int m2 = 2 * M - 1, M2 = 2 * M;
    unsigned long long n_rolled = 0;

    // the n windows of a canonical record into the k-mer table (as k_skbucket's roll_out)
    auto roll_out = [&](uint32_t x0, uint32_t x1, uint32_t x2, unsigned int mult, unsigned int ea, unsigned int eb) {
        const unsigned int n = (x2 >> 28) + 1;
        if (dbg) n_rolled += n;
        auto events = [&](uint64_t fwd, uint64_t rc, unsigned int o, unsigned int &eC, unsigned int &eT,
                          unsigned int &add) {
            const bool tw = fwd > rc;
            const unsigned int ef = ea + o, et = eb - o;
            add = mult;
            eC = tw ? et : ef;
            eT = tw ? ef : et;
            if (EVEN_K && fwd == rc) {
                add = 2 * mult;
                eC = eT = min(ef, et);
            }
            return tw ? rc : fwd;
        };
        const unsigned int h = (n + 1) >> 1;
        auto at = [&](unsigned int o, uint64_t &fw, uint64_t &rv) {
            const uint32_t lo = __builtin_amdgcn_alignbit(x1, x0, 2 * o), hi = __builtin_amdgcn_alignbit(x2, x1, 2 * o);
            const uint64_t P = (uint64_t)lo | (uint64_t)hi << 32;
            rv = ~P & kmask;
            fw = rev2_64(P) >> fsh;
        };
        auto roll = [&](unsigned int o, uint64_t &fw, uint64_t &rv) {
            const unsigned int tb = o + (unsigned int)k - 1;
            const uint32_t wd = tb < 32 ? x1 : x2;
            const uint32_t bb = (wd >> (2 * (tb & 15))) & 3u;
            fw = ((fw << 2) | bb) & kmask;
            rv = (rv >> 2) | ((uint64_t)(3u - bb) << sh);
        };
        uint64_t fA, rA, fB, rB;
        at(0, fA, rA);
        at(h, fB, rB);
        for (unsigned int i = 0; i < h; i++) {
            const unsigned int oB = i + h;
            const bool bB = oB < n;
            if (i) {
                roll(i, fA, rA);
                roll(oB, fB, rB);
            }
            unsigned int eCA, eTA, eCB, eTB, addA, addB;
            const uint64_t cA = events(fA, rA, i, eCA, eTA, addA);
            const uint64_t cB = events(fB, rB, oB, eCB, eTB, addB);
            unsigned int sA = (sk_slot(cA) >> (32 - SBITS)) & (SLOTS - 1), sB = (sk_slot(cB) >> (32 - SBITS)) & (SLOTS - 1);
            const unsigned long long kA = tab.key[sA], kB = tab.key[sB];
            lds_locate2<SLOTS>(tab, s_over, cA, sA, kA, cB, sB, bB ? kB : cB);
            atomicAdd(&tab.count[sA], addA);
            if (bB) atomicAdd(&tab.count[sB], addB);
            const uint2 vA = tab.ev[sA], vB = tab.ev[sB];
            if (eCA < vA.x) atomicMin(&tab.ev[sA].x, eCA);
            if (eTA < vA.y) atomicMin(&tab.ev[sA].y, eTA);
            if (bB && eCB < vB.x) atomicMin(&tab.ev[sB].x, eCB);
            if (bB && eTB < vB.y) atomicMin(&tab.ev[sB].y, eTB);
        }
    };

    // ---- records -> record table (k_skbucket's protocol; PD rounds of loads in flight) --------
    constexpr int PD = SK2_PD;
    uint4 nx[PD];
#pragma unroll
    for (int d = 0; d < PD; d++) nx[d] = recs[r1 > r0 ? min(r0 + tid + (uint64_t)d * NT, r1 - 1) : r0];
    auto ld = [](uint32_t *a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto record_round = [&](uint4 &nxd, uint64_t c0) {
        const uint64_t ri = c0 + tid;
        const bool valid = ri < r1;
        const uint4 x = nxd;
        nxd = recs[min(ri + PD * NT, r1 - 1)];
        const unsigned int n = (x.z >> 28) + 1, L2 = 2 * (n + (unsigned int)k - 1);
        const uint32_t m1 = L2 >= 64 ? 0xFFFFFFFFu : (1u << ((L2 - 32) & 31)) - 1u;
        const uint32_t mw2 = L2 > 64 ? (1u << ((L2 - 64) & 31)) - 1u : 0u;
        const uint32_t x0 = x.x, x1 = x.y & m1, x2 = x.z & mw2;
        const uint32_t y0 = rev2_32b(x2), y1 = rev2_32b(x1), y2 = rev2_32b(x0);
        const unsigned int sft = 96 - L2, s5 = sft & 31;
        const bool lo = sft < 32;
        const uint32_t a0 = __builtin_amdgcn_alignbit(y1, y0, s5), a1 = __builtin_amdgcn_alignbit(y2, y1, s5),
                       a2 = y2 >> s5;
        const uint32_t q0 = ~(lo ? a0 : a1), q1 = ~(lo ? a1 : a2) & m1, q2 = lo ? ~a2 & mw2 : 0u;
        const bool flip = q2 != x2 ? q2 < x2 : q1 != x1 ? q1 < x1 : q0 < x0;
        const unsigned int p = x.w;
        const unsigned int rd0 = (unsigned int)((double)p * inv_m);
        int rm = (int)(p - rd0 * M);
        unsigned int rd = rd0;
        if (rm < 0) rd--, rm += (int)M;
        else if (rm >= (int)M) rd++, rm -= (int)M;
        const unsigned int A = rd * M2 + (unsigned int)rm, B = rd * M2 + m2 - (unsigned int)rm;
        const uint32_t K0 = flip ? q0 : x0, K1 = flip ? q1 : x1, K2 = (flip ? q2 : x2) | (n - 1) << 28;
        const uint32_t EA = flip ? B - n + 1 : A, EB = flip ? A + n - 1 : B;
        uint32_t hh = K0 * 0x9E3779B1u;
        hh = (hh ^ (hh >> 15) ^ K1) * 0x85EBCA77u;
        hh = (hh ^ (hh >> 13) ^ K2) * 0xC2B2AE3Du;
        hh ^= hh >> 16;
        const uint32_t TG = (hh | 0x1000u) & 0xFFFFF000u;
        uint32_t SL = __umulhi(hh * 0x27D4EB2Fu, (unsigned int)RS);
        int ST = valid ? 0 : 1;  // 0 searching, 1 found / claimed, 2 past the claim cap
#pragma unroll 1
        while (__any(ST == 0)) {
            const uint32_t T = ld(&R.tag[SL]);
            asm volatile("" ::: "memory");  // the key words are read after the tag (issue order)
            const uint32_t X = ld(&R.x[SL]), Y = ld(&R.y[SL]), Z = ld(&R.z[SL]);
            const bool hit = T == TG && X == K0 && Y == K1 && Z == K2;
            const bool go = ST == 0;
            ST = go && hit ? 1 : ST;
            const bool claim = go && !hit && T == 0;
            if (go && !hit && T != 0 && T != (TG | PEND)) SL = SL + 1 == (unsigned int)RS ? 0u : SL + 1;
            if (claim) {
                // reserve an entry first, so the table never holds more than the cap (the compact
                // arrays below hold NC = RS / 2 entries): a lane past it, or one whose CAS loses,
                // gives its reservation back (claim_cap: tests of the overflow list)
                const unsigned int o = atomicAdd(&s_nent, 1u);
                if (o >= min(CLAIM_MAX, claim_cap)) {
                    atomicSub(&s_nent, 1u);
                    ST = 2;
                } else if (atomicCAS(&R.tag[SL], 0u, TG | PEND) == 0) {
                    R.x[SL] = K0, R.y[SL] = K1, R.z[SL] = K2;
                    __hip_atomic_store(&R.tag[SL], TG, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    ST = 1;
                } else {
                    atomicSub(&s_nent, 1u);
                }
            }
        }
        if (valid && ST == 1) {
            atomicAdd(&R.mult[SL], 1u);
            if (EA < R.a[SL]) atomicMin(&R.a[SL], EA);
            if (EB < R.b[SL]) atomicMin(&R.b[SL], EB);
        }
        if (ST == 2) {  // the overflow list (full: the call is redone elsewhere)
            const unsigned int o = atomicAdd(&s_nov, 1u);
            if (o < (unsigned int)OV) o_x[o] = K0, o_y[o] = K1, o_z[o] = K2, o_a[o] = EA, o_b[o] = EB;
            else s_over[0] = 1;
        }
    };
    for (uint64_t c0 = r0; c0 < r1; c0 += PD * NT) {
#pragma unroll
        for (int d = 0; d < PD; d++) {
            if (c0 + (uint64_t)d * NT >= r1) break;  // uniform
            record_round(nx[d], c0 + (uint64_t)d * NT);
        }
    }
    __syncthreads();
    // ---- distinct records out of the record table, counted by window count --------------------
    constexpr int PER = (RS + NT - 1) / NT;
    uint32_t cx[PER], cy[PER], cz[PER], cm[PER], ca[PER], cb[PER], bin[PER], rk[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const unsigned int i = tid + q * NT;
        bin[q] = SK2_NMAX;
        if (i < (unsigned)RS && R.tag[i]) {
            cx[q] = R.x[i], cy[q] = R.y[i], cz[q] = R.z[i], cm[q] = R.mult[i], ca[q] = R.a[i], cb[q] = R.b[i];
            bin[q] = SK2_NMAX - 1 - (cz[q] >> 28);  // most windows first
            rk[q] = atomicAdd(&s_ncnt[bin[q]], 1u);
        }
    }
    __syncthreads();
    if (tid == 0) {
        unsigned int a = 0;
        for (int q = 0; q < SK2_NMAX; q++) {
            const unsigned int v = s_ncnt[q];
            s_ncnt[q] = a;
            a += v;
        }
        s_ncnt[SK2_NMAX] = a;
        if (dbg) {
            atomicAdd(&dbg[0], (unsigned long long)a), atomicAdd(&dbg[1], 1ull);
            atomicMax(&dbg[3], (unsigned long long)(a + min(s_nov, (unsigned int)OV)));  // distinct, overflow incl.
        }
    }
    // the k-mer table over the record table's space (its reads are done)
    for (int i = tid; i < SLOTS; i += NT) {
        tab.key[i] = EMPTY_KEY;
        tab.count[i] = 0;
        tab.ev[i] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++)
        if (bin[q] < SK2_NMAX) {
            const unsigned int o = s_ncnt[bin[q]] + rk[q];
            L.k.x[o] = cx[q], L.k.y[o] = cy[q], L.k.z[o] = cz[q], L.k.mult[o] = cm[q], L.k.a[o] = ca[q], L.k.b[o] = cb[q];
        }
    __syncthreads();
    const unsigned int ne = s_ncnt[SK2_NMAX], nov = min(s_nov, (unsigned int)OV);
    for (unsigned int t = tid; t < ne + nov; t += NT) {
        if (t < ne) roll_out(L.k.x[t], L.k.y[t], L.k.z[t], L.k.mult[t], L.k.a[t], L.k.b[t]);
        else {
            const unsigned int o = t - ne;
            roll_out(o_x[o], o_y[o], o_z[o], 1u, o_a[o], o_b[o]);
        }
    }
    if (dbg) atomicAdd(&dbg[2], n_rolled);
    lds_table_finish<SLOTS, false, KeyId, LTabE<SLOTS>, EvExpand, NT>(tab, s_over, b, limit, dkey, dcnt, dfc, dft, sub,
                                                                      nsolid, ndistinct, overflow, KeyId(),
                                                                      EvExpand{2 * M}, bmark);
}


// ---- error-rich input: super-k-mer buckets behind a seen-twice filter (round 4) ----------------
// With sequencing errors most distinct k-mers occur once (ecoli10m_err: 1.6e8 distinct, 1.3e7
// solid) and a bucket's records are mostly unique, so k_skbucket3's record merge finds nothing
// to merge and its tables would overflow.  Here every record's windows are rolled out twice, as
// k_bucket_filt (count_part.h) does for window records: pass 0 marks two cells per canonical
// key in LDS bitmaps (seen once / seen twice); pass 1 inserts a window only if both of its
// cells were seen twice (every key occurring >= 2 times passes; a singleton passes with the
// probability of a double cell collision, and is then counted exactly and dropped by the solid
// filter) or if its own insert already exceeds the limit (an even-k palindrome adds 2).  The
// table holds the bucket's solid keys plus those few singletons; a bucket whose twice-seen
// cells estimate more keys than the table takes reports an overflow (the call is redone on
// window records).  Requires limit >= 1 (with limit < 1 every key is solid).
// 2^17 cells a bitmap (2 x 16 KiB of LDS beside the 40 KiB table: two workgroups per CU).  At the
// error-rich headline (~9800 distinct keys, ~800 solid a bucket) a singleton passes with
// p^2, p = 1 - exp(-2D/m) = 0.14: ~170 singletons a table; 2^16 cells passed ~600 and overflowed
// the 1474-key budget in many buckets
constexpr int SKF_BITS = 17;  // filter cells per bitmap
// MERGED (round 5): the bucket's records merged by k_skdedup first -- {canonical bases | (n - 1)
// << 28, multiplicity} with their event minima {A, B} in mev -- so a super-k-mer read ~130 times
// rolls out its windows once, with add = multiplicity (a key of a record seen twice is repeated:
// its cells are marked seen twice at once, and it is inserted without the filter's test)
template <int SLOTS, int NT, bool EVEN_K, bool MERGED = false>
__global__ void __launch_bounds__(NT) k_skbucket_filt(const uint4 *recs, const unsigned long long *bbeg,
                                                      const unsigned long long *bend, int k, uint32_t M, double inv_m,
                                                      long long limit, unsigned long long *dkey, unsigned int *dcnt,
                                                      unsigned long long *dfc, unsigned long long *dft, SubSlot *sub,
                                                      unsigned int *nsolid, unsigned long long *ndistinct,
                                                      unsigned int *overflow, unsigned int max_keys,
                                                      unsigned long long *dbg = nullptr, unsigned int *bmark = nullptr,
                                                      const uint2 *mev = nullptr) {
    constexpr int SBITS = __builtin_ctz(SLOTS);
    constexpr unsigned int NW = 1u << (SKF_BITS - 5), CM = (1u << SKF_BITS) - 1;
    __shared__ LTabE<SLOTS> tab;
    __shared__ unsigned int s_over[2];
    __shared__ unsigned int seen1[NW], seen2[NW];
    __shared__ unsigned int s_cells[2];
    const unsigned int b = blockIdx.x, tid = threadIdx.x;
    for (int i = tid; i < SLOTS; i += NT) {
        tab.key[i] = EMPTY_KEY;
        tab.count[i] = 0;
        tab.ev[i] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    }
    for (unsigned int i = tid; i < NW; i += NT) seen1[i] = seen2[i] = 0;
    if (tid == 0) s_over[0] = s_over[1] = 0, s_cells[0] = s_cells[1] = 0;
    __syncthreads();
    const uint64_t r0 = bbeg[b], r1 = bend[b];
    const uint64_t kmask = kmask64(k);
    const int fsh = 64 - 2 * k;
    const unsigned int m2 = 2 * M - 1, M2 = 2 * M;
    // the windows of a record as stored (window o = bases o .. o + k - 1, o < n <= 16): canonical
    // key, add, first events of the canonical / twin string (k_skbucket3's roll-out, unflipped)
    auto windows = [&](uint64_t ri, const uint4 &x, auto &&fn) {
        const unsigned int n = (x.z >> 28) + 1;
        if constexpr (MERGED) {  // canonical record: window o at A + o, its twin at B - o
            const uint2 e = mev[ri];
            const unsigned int mult = x.w;
            for (unsigned int o = 0; o < n; o++) {
                const uint32_t lo = __builtin_amdgcn_alignbit(x.y, x.x, 2 * o), hi = __builtin_amdgcn_alignbit(x.z, x.y, 2 * o);
                const uint64_t P = (uint64_t)lo | (uint64_t)hi << 32;
                const uint64_t rv = ~P & kmask, fw = rev2_64(P) >> fsh;
                const bool tw = fw > rv;
                const unsigned int ef = e.x + o, et = e.y - o;
                unsigned int add = mult, eC = tw ? et : ef, eT = tw ? ef : et;
                if (EVEN_K && fw == rv) {
                    add = 2 * mult;
                    eC = eT = min(ef, et);
                }
                fn(tw ? rv : fw, add, eC, eT);
            }
            return;
        }
        const unsigned int p = x.w;
        const unsigned int rd0 = (unsigned int)((double)p * inv_m);
        int rm = (int)(p - rd0 * M);
        unsigned int rd = rd0;
        if (rm < 0) rd--, rm += (int)M;
        else if (rm >= (int)M) rd++, rm -= (int)M;
        const unsigned int A = rd * M2 + (unsigned int)rm, B = rd * M2 + m2 - (unsigned int)rm;
        for (unsigned int o = 0; o < n; o++) {
            const uint32_t lo = __builtin_amdgcn_alignbit(x.y, x.x, 2 * o), hi = __builtin_amdgcn_alignbit(x.z, x.y, 2 * o);
            const uint64_t P = (uint64_t)lo | (uint64_t)hi << 32;
            const uint64_t rv = ~P & kmask, fw = rev2_64(P) >> fsh;
            const bool tw = fw > rv;
            const unsigned int ef = A + o, et = B - o;
            unsigned int add = 1, eC = tw ? et : ef, eT = tw ? ef : et;
            if (EVEN_K && fw == rv) {
                add = 2;
                eC = eT = min(ef, et);
            }
            fn(tw ? rv : fw, add, eC, eT);
        }
    };
    auto cells = [](unsigned long long c, unsigned int &c1, unsigned int &c2) {
        const uint64_t h = mix64(c);
        c1 = (unsigned int)(h >> 12) & CM;
        c2 = (unsigned int)(h >> 30) & CM;
    };
    // pass 0: the filter
    for (uint64_t i = r0 + tid; i < r1; i += NT) {
        const uint4 x = recs[i];
        const bool rep = MERGED && x.w > 1;  // (a merged record seen twice: its keys are repeated)
        windows(i, x, [&](unsigned long long c, unsigned int, unsigned int, unsigned int) {
            unsigned int c1, c2;
            cells(c, c1, c2);
            const unsigned int m1 = 1u << (c1 & 31), mm2 = 1u << (c2 & 31);
            if (rep) {
                atomicOr(&seen1[c1 >> 5], m1), atomicOr(&seen2[c1 >> 5], m1);
                atomicOr(&seen1[c2 >> 5], mm2), atomicOr(&seen2[c2 >> 5], mm2);
                return;
            }
            if (atomicOr(&seen1[c1 >> 5], m1) & m1) atomicOr(&seen2[c1 >> 5], m1);
            if (atomicOr(&seen1[c2 >> 5], mm2) & mm2) atomicOr(&seen2[c2 >> 5], mm2);
        });
    }
    __syncthreads();
    {  // keys that will be inserted, and the bucket's distinct keys, by linear counting
        unsigned int n2 = 0, n1 = 0;
        for (unsigned int i = tid; i < NW; i += NT) n2 += __popc(seen2[i]), n1 += __popc(seen1[i]);
        for (int o = 32; o > 0; o >>= 1) n2 += __shfl_down(n2, o), n1 += __shfl_down(n1, o);
        if ((tid & 63) == 0) atomicAdd(&s_cells[0], n2), atomicAdd(&s_cells[1], n1);
        __syncthreads();
        if (tid == 0) {
            // D distinct keys (linear counting on the seen-once cells, 2 marks a key); the
            // seen-twice cells beyond those of random collisions, m (1 - e^-l (1 + l)), l = 2D/m,
            // are ~2 per repeated key S; a singleton passes when both its cells hold another
            // mark, (1 - e^-l)^2: the table receives S + (D - S) (1 - e^-l)^2 keys
            const double m = (double)(1u << SKF_BITS);
            const double D = -m * log(1.0 - (double)min(s_cells[1], CM) / m) / 2.0;
            const double l = 2.0 * D / m, el = exp(-l);
            const double S = fmax(0.0, ((double)s_cells[0] - m * (1.0 - el * (1.0 + l))) / 2.0);
            const double pass = 1.1 * (S + fmax(0.0, D - S) * (1.0 - el) * (1.0 - el));  // (~10 % low: solid cells hit by collisions)
            if (pass > (double)max_keys) s_over[0] = 1;  // (default 1900 of the table's 2048 slots)
            else atomicAdd(ndistinct, (unsigned long long)llround(D));
            if (dbg) {  // EULERHIP_SK2_STATS: the largest estimates, the predictor's refusals
                atomicMax(&dbg[0], (unsigned long long)D);
                atomicMax(&dbg[1], (unsigned long long)pass);
                atomicMax(&dbg[2], (unsigned long long)s_cells[0]);
                atomicMax(&dbg[3], (unsigned long long)(bend[b] - bbeg[b]));
                if (s_over[0]) atomicAdd(&dbg[4], 1ull);
            }
        }
        __syncthreads();
    }
    if (s_over[0]) {
        if (tid == 0) atomicAdd(overflow, 1u);
        return;
    }
    // pass 1: the keys seen twice (or solid by their own insert) into the table
    for (uint64_t i = r0 + tid; i < r1; i += NT) {
        windows(i, recs[i], [&](unsigned long long c, unsigned int add, unsigned int eC, unsigned int eT) {
            if ((long long)add <= limit) {  // (add > limit: solid by this insert alone)
                unsigned int c1, c2;
                cells(c, c1, c2);
                const bool twice = ((seen2[c1 >> 5] >> (c1 & 31)) & (seen2[c2 >> 5] >> (c2 & 31)) & 1u) != 0;
                if (!twice) return;
            }
            const unsigned int s0 = (sk_slot(c) >> (32 - SBITS)) & (SLOTS - 1);
            const unsigned int sl = lds_locate<SLOTS>(tab, s_over, c, s0, tab.key[s0]);
            atomicAdd(&tab.count[sl], add);
            const uint2 v = tab.ev[sl];
            if (eC < v.x) atomicMin(&tab.ev[sl].x, eC);
            if (eT < v.y) atomicMin(&tab.ev[sl].y, eT);
        });
    }
    if (dbg) {
        __syncthreads();
        if (tid == 0) {
            if (s_over[0]) atomicAdd(&dbg[5], 1ull);  // tables that filled up in pass 1
            atomicMax(&dbg[6], (unsigned long long)s_over[1]);  // most keys inserted
        }
    }
    lds_table_finish<SLOTS, false, KeyId, LTabE<SLOTS>, EvExpand, NT>(tab, s_over, b, limit, dkey, dcnt, dfc, dft, sub,
                                                                      nsolid, nullptr, overflow, KeyId(),
                                                                      EvExpand{2 * M}, bmark);
}


// ---- error-rich input: the bucket's duplicate records merged in front of the filter (round 5) -----
// At 0.5 % substitutions ~60 % of the reads are error-free and most super-k-mers of the others
// are too: ecoli10m_err's buckets hold ~6300 records of which ~1200 are distinct.  k_skdedup merges
// a bucket's records by canonical content (k_skbucket3's record table and claim protocol) and
// writes the distinct ones -- {bases | (n - 1) << 28, multiplicity} + {A, B} -- at the bucket's
// start in mrec / mev; a record past the table's claim cap is written as it is (multiplicity 1,
// any split of the copies between entries is exact).  k_skbucket_filt<MERGED> then rolls out
// ~6x fewer windows, twice.  mend[b] = the end of bucket b's merged records.  (Round 4 merged in
// the filter kernel itself: its 131 KB of LDS held one workgroup per CU, slower than no merge.)
template <int RS, int NT>
__global__ void __launch_bounds__(NT) k_skdedup(const uint4 *recs, const unsigned long long *bbeg,
                                                const unsigned long long *bend, int k, uint32_t M, double inv_m,
                                                uint4 *mrec, uint2 *mev, unsigned long long *mend,
                                                unsigned int claim_cap = ~0u, unsigned long long *dbg = nullptr) {
    constexpr uint32_t PEND = 0x800u;
    constexpr unsigned int CLAIM_MAX = RS - 1 - NT;  // (probes of the records in flight end)
    static_assert(RS > NT + 1, "record table too small for the records in flight");
    __shared__ uint32_t tag[RS], tx[RS], ty[RS], tz[RS], tm[RS], ta[RS], tb[RS];
    __shared__ unsigned int s_nent, s_nout, s_nrej, s_ncnt[SK2_NMAX];
    const unsigned int b = blockIdx.x, tid = threadIdx.x;
    for (int i = tid; i < RS; i += NT) {
        tag[i] = 0;
        tm[i] = 0;
        ta[i] = tb[i] = 0xFFFFFFFFu;
    }
    if (tid == 0) s_nent = 0, s_nout = 0, s_nrej = 0;
    if (tid < (unsigned int)SK2_NMAX) s_ncnt[tid] = 0;
    __syncthreads();
    const uint64_t r0 = bbeg[b], r1 = bend[b];
    const unsigned int m2 = 2 * M - 1, M2 = 2 * M;
    auto ld = [](uint32_t *a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    // (the next round's record loaded before this round's probes: one load in flight per
    // thread left the kernel waiting on HBM latency)
    uint4 nxt = r1 > r0 ? recs[min(r0 + tid, r1 - 1)] : make_uint4(0u, 0u, 0u, 0u);
    for (uint64_t c0 = r0; c0 < r1; c0 += NT) {
        const uint64_t ri = c0 + tid;
        const bool valid = ri < r1;
        const uint4 x = nxt;
        if (c0 + NT < r1) nxt = recs[min(ri + NT, r1 - 1)];
        // canonical content (k_skbucket3's record round)
        const unsigned int n = (x.z >> 28) + 1, L2 = 2 * (n + (unsigned int)k - 1);
        const uint32_t m1 = L2 >= 64 ? 0xFFFFFFFFu : (1u << ((L2 - 32) & 31)) - 1u;
        const uint32_t mw2 = L2 > 64 ? (1u << ((L2 - 64) & 31)) - 1u : 0u;
        const uint32_t x0 = x.x, x1 = x.y & m1, x2 = x.z & mw2;
        const uint32_t y0 = rev2_32b(x2), y1 = rev2_32b(x1), y2 = rev2_32b(x0);
        const unsigned int sft = 96 - L2, s5 = sft & 31;
        const bool lo = sft < 32;
        const uint32_t a0 = __builtin_amdgcn_alignbit(y1, y0, s5), a1 = __builtin_amdgcn_alignbit(y2, y1, s5),
                       a2 = y2 >> s5;
        const uint32_t q0 = ~(lo ? a0 : a1), q1 = ~(lo ? a1 : a2) & m1, q2 = lo ? ~a2 & mw2 : 0u;
        const bool flip = q2 != x2 ? q2 < x2 : q1 != x1 ? q1 < x1 : q0 < x0;
        const unsigned int p = x.w;
        const unsigned int rd0 = (unsigned int)((double)p * inv_m);
        int rm = (int)(p - rd0 * M);
        unsigned int rd = rd0;
        if (rm < 0) rd--, rm += (int)M;
        else if (rm >= (int)M) rd++, rm -= (int)M;
        const unsigned int A = rd * M2 + (unsigned int)rm, B = rd * M2 + m2 - (unsigned int)rm;
        const uint32_t K0 = flip ? q0 : x0, K1 = flip ? q1 : x1, K2 = (flip ? q2 : x2) | (n - 1) << 28;
        const uint32_t EA = flip ? B - n + 1 : A, EB = flip ? A + n - 1 : B;
        uint32_t hh = K0 * 0x9E3779B1u;
        hh = (hh ^ (hh >> 15) ^ K1) * 0x85EBCA77u;
        hh = (hh ^ (hh >> 13) ^ K2) * 0xC2B2AE3Du;
        hh ^= hh >> 16;
        const uint32_t TG = (hh | 0x1000u) & 0xFFFFF000u;
        uint32_t SL = __umulhi(hh * 0x27D4EB2Fu, (unsigned int)RS);
        int ST = valid ? 0 : 1;  // 0 searching, 1 found / claimed, 2 past the claim cap
#pragma unroll 1
        while (__any(ST == 0)) {
            const uint32_t T = ld(&tag[SL]);
            asm volatile("" ::: "memory");  // the key words are read after the tag (issue order)
            const uint32_t X = ld(&tx[SL]), Y = ld(&ty[SL]), Z = ld(&tz[SL]);
            const bool hit = T == TG && X == K0 && Y == K1 && Z == K2;
            const bool go = ST == 0;
            ST = go && hit ? 1 : ST;
            const bool claim = go && !hit && T == 0;
            if (go && !hit && T != 0 && T != (TG | PEND)) SL = SL + 1 == (unsigned int)RS ? 0u : SL + 1;
            if (claim) {
                const unsigned int o = atomicAdd(&s_nent, 1u);
                if (o >= min(CLAIM_MAX, claim_cap)) {  // (claim_cap: tests of the records past the cap)
                    atomicSub(&s_nent, 1u);
                    ST = 2;
                } else if (atomicCAS(&tag[SL], 0u, TG | PEND) == 0) {
                    tx[SL] = K0, ty[SL] = K1, tz[SL] = K2;
                    __hip_atomic_store(&tag[SL], TG, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    ST = 1;
                } else {
                    atomicSub(&s_nent, 1u);
                }
            }
        }
        if (valid && ST == 1) {
            atomicAdd(&tm[SL], 1u);
            if (EA < ta[SL]) atomicMin(&ta[SL], EA);
            if (EB < tb[SL]) atomicMin(&tb[SL], EB);
        }
        if (ST == 2) {  // past the cap: written on its own
            if (dbg) atomicAdd(&s_nrej, 1u);
            const uint64_t o = r0 + atomicAdd(&s_nout, 1u);
            mrec[o] = make_uint4(K0, K1, K2, 1u);
            mev[o] = make_uint2(EA, EB);
        }
    }
    __syncthreads();
    // the distinct records out by window count, most windows first (after those past the cap):
    // the filter rolls a record's windows out in one lane, so a wave of mixed counts ran at the
    // pace of its longest record (~42 % of its lanes busy on ecoli10m_err)
    constexpr int PER = (RS + NT - 1) / NT;
    uint32_t bin[PER], rk[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const unsigned int i = tid + q * NT;
        bin[q] = SK2_NMAX;
        if (i < (unsigned int)RS && tag[i]) {
            bin[q] = SK2_NMAX - 1 - (tz[i] >> 28);
            rk[q] = atomicAdd(&s_ncnt[bin[q]], 1u);
        }
    }
    __syncthreads();
    if (tid == 0) {
        unsigned int a = s_nout;  // (the records past the cap come first)
        for (int q = 0; q < SK2_NMAX; q++) {
            const unsigned int v = s_ncnt[q];
            s_ncnt[q] = a;
            a += v;
        }
        s_nout = a;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
        if (bin[q] == SK2_NMAX) continue;
        const unsigned int i = tid + q * NT;
        const uint64_t o = r0 + s_ncnt[bin[q]] + rk[q];
        mrec[o] = make_uint4(tx[i], ty[i], tz[i], tm[i]);
        mev[o] = make_uint2(ta[i], tb[i]);
    }
    __syncthreads();
    if (tid == 0) {
        mend[b] = r0 + s_nout;
        if (dbg) {  // EULERHIP_SK2_STATS: most merged records / records past the cap a bucket, all merged
            atomicMax(&dbg[7], (unsigned long long)s_nout);
            atomicMax(&dbg[8], (unsigned long long)s_nrej);
            atomicAdd(&dbg[9], (unsigned long long)s_nout);
        }
    }
}

}  // namespace ec
