// window.h -- read access and the reference-order k-mer window iterator (build:27-35).
#pragma once
#include "common.h"

namespace ec {
constexpr int HLL_BITS = 12;
constexpr int HLL_M = 1 << HLL_BITS;
constexpr int MAX_PROBE = 1 << 14;

// sequential byte reader over aligned 32-bit words (an aligned word never crosses a page,
// so reading the word that holds a valid byte is always in-bounds of the allocation)
struct ByteReader {
    uint64_t base;  // absolute address of byte 0
    uint64_t wpos;
    uint32_t word;
    __device__ ByteReader(const uint8_t *b) : base((uint64_t)b), wpos(~0ull), word(0) {}
    __device__ inline uint32_t operator()(uint64_t pos) {
        const uint64_t addr = base + pos;
        const uint64_t a = addr & ~3ull;
        if (a != wpos) {
            wpos = a;
            word = *reinterpret_cast<const uint32_t *>(a);
        }
        return (word >> ((addr & 3) * 8)) & 0xFFu;
    }
};

// Iterate the windows of read r in reference insertion order (build:27-35).  For every
// valid window calls fn(fwd, rc, ef, er): fwd/rc = 2-bit codes of the window and of its
// twin, ef/er = the dict insertion events of the forward string (build:31-32) and of the
// twin string (build:33-35, window j of twin(seg) is the twin of forward window m-1-j).
// Event = (read << 32) | local, local = 2*wb + i (forward) or 2*wb + 2m-1-i (twin).
template <typename Reader, typename Fn>
__device__ inline uint32_t for_each_window(Reader &rd, uint64_t s, uint64_t len, int k,
                                           uint64_t r, Fn &&fn) {
    const uint64_t mask = kmask64(k);
    const int sh = 2 * (k - 1);
    uint32_t wb = 0;
    uint64_t p = 0;
    while (p < len) {
        uint64_t q = p;
        while (q < len && base_code(rd(s + q)) < 4) q++;
        if (q - p >= (uint64_t)k) {
            const uint32_t m = (uint32_t)(q - p - k + 1);
            uint64_t fwd = 0, rc = 0;
            for (uint64_t t = p; t < q; t++) {
                const uint64_t b = base_code(rd(s + t));
                fwd = ((fwd << 2) | b) & mask;
                rc = (rc >> 2) | ((3ull - b) << sh);
                if (t - p + 1 >= (uint64_t)k) {
                    const uint32_t i = (uint32_t)(t - p + 1 - k);
                    const uint64_t ef = (r << 32) | (uint64_t)(2 * wb + i);
                    const uint64_t er = (r << 32) | (uint64_t)(2 * wb + 2 * m - 1 - i);
                    fn(fwd, rc, ef, er);
                }
            }
            wb += m;
        }
        p = q + 1;
    }
    return wb;
}

// ---- branch-free fast path for reads over {A,C,G,T} only ------------------------------
// 2-bit code of an ASCII base; equals the reference table codeF[c & 7] (src/pyencode.py:40)
// on A, C, G, T.
__device__ inline uint32_t code2(uint32_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }
__device__ inline uint32_t is_acgt(uint32_t c) {
    return (uint32_t)((c & 0xE0u) == 0x40u) & ((0x0010008Au >> (c & 31u)) & 1u);
}

// A read staged in LDS, read 4 bytes at a time: chunk(i) = read bytes 4i..4i+3 (little
// endian), built from two dword LDS loads and one v_alignbyte whatever the read's alignment.
struct LdsRead {
    const uint32_t *w;
    uint32_t d0;  // dword index holding the read's first byte
    uint32_t sh;  // its byte offset within that dword
    __device__ inline uint32_t chunk(uint32_t i) const {
        return __builtin_amdgcn_alignbyte(w[d0 + i + 1], w[d0 + i], sh);
    }
};

// bit 0: read has an 'N'; bit 1: read has a byte outside {A,C,G,T,N}
__device__ inline uint32_t read_flags(const LdsRead &rv, uint32_t len) {
    uint32_t nn = 0, bad = 0;
    const uint32_t full = len >> 2;
    for (uint32_t i = 0; i < full; i++) {
        const uint32_t c4 = rv.chunk(i);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t c = (c4 >> (8 * q)) & 0xFFu;
            const uint32_t n = c == 'N';
            nn |= n;
            bad |= (is_acgt(c) | n) ^ 1u;
        }
    }
    if (len & 3) {
        const uint32_t c4 = rv.chunk(full);
        for (uint32_t q = 0; q < (len & 3); q++) {
            const uint32_t c = (c4 >> (8 * q)) & 0xFFu;
            const uint32_t n = c == 'N';
            nn |= n;
            bad |= (is_acgt(c) | n) ^ 1u;
        }
    }
    return nn | (bad << 1);
}

// Windows of an N-free read (one segment, wb = 0, m = len-k+1): fn(fwd, rc, i) for i < m;
// the insertion events are i (forward string) and 2m-1-i (twin string), as in for_each_window.
// HI (k >= 17): both rolls touch only the high word for the mask / the entering twin base.
template <bool HI, typename Fn>
__device__ inline void windows_clean_t(const LdsRead &rv, uint32_t len, int k, Fn &&fn) {
    const uint64_t mask = kmask64(k);
    const uint32_t mhi = (uint32_t)(mask >> 32);
    const int sh = 2 * (k - 1);
    uint64_t fwd = 0, rc = 0;
    const uint32_t km1 = (uint32_t)(k - 1);
    auto roll = [&](uint32_t b) {
        if (HI) {
            fwd = (fwd << 2) | b;
            fwd &= ((uint64_t)mhi << 32) | 0xFFFFFFFFull;
            rc = (rc >> 2) | ((uint64_t)((3u - b) << (sh - 32)) << 32);
        } else {
            fwd = ((fwd << 2) | b) & mask;
            rc = (rc >> 2) | ((uint64_t)(3u - b) << sh);
        }
    };
    const uint32_t full = len >> 2;
    for (uint32_t i = 0; i < full; i++) {
        const uint32_t c4 = rv.chunk(i);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            roll(code2(c4 >> (8 * q)));
            const uint32_t t = 4 * i + q;
            if (t >= km1) fn(fwd, rc, t - km1);
        }
    }
    if (len & 3) {
        const uint32_t c4 = rv.chunk(full);
        for (uint32_t q = 0; q < (len & 3); q++) {
            roll(code2(c4 >> (8 * q)));
            const uint32_t t = 4 * full + q;
            if (t >= km1) fn(fwd, rc, t - km1);
        }
    }
}
template <typename Fn>
__device__ inline void windows_clean(const LdsRead &rv, uint32_t len, int k, Fn &&fn) {
    if (k >= 17)
        windows_clean_t<true>(rv, len, k, fn);
    else
        windows_clean_t<false>(rv, len, k, fn);
}

}  // namespace ec
