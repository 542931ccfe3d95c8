// hostin.h -- device side of the host-input path (ec_assemble_host, ec_assemble_packed_host).
//
// The reference's GPU path starts from reads in host memory (src/eulercuda.py:484-497: the
// read buffer goes to encode_lmer_device and is copied H2D there).  Here the host reads reach
// HBM in chunks on a copy stream while the session stream already partitions the chunks that
// have arrived (assemble.hip pipe_upto).  Reads come as ASCII (ec_assemble_host) or 2 bits per
// base (ec_assemble_packed_host, a quarter of the PCIe bytes): k_unpack2 expands a chunk of
// codes to the ASCII layout every count kernel reads, k_patch restores the bytes that are not
// A/C/G/T (N and anything else: the count path then treats them as it treats ASCII input).
#pragma once
#include "common.h"

namespace ec {

// bases [blo, bhi) of the 2-bit stream (base i at bits 2 (i & 15) of word i >> 4) -> ASCII
// out[blo .. bhi); one thread per 16 bases (one 32-bit load, one 16-byte store)
__global__ void __launch_bounds__(256) k_unpack2(const uint32_t *__restrict__ codes, uint64_t blo, uint64_t bhi,
                                                 uint8_t *__restrict__ out) {
    const uint64_t u0 = blo >> 4, u1 = (bhi + 15) >> 4;
    for (uint64_t u = u0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < u1;
         u += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t w = codes[u];
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t x = (w >> (8 * q)) & 0xFFu;  // 4 codes -> one selector byte each
            const uint32_t sel = (x & 3u) | ((x & 0xCu) << 6) | ((x & 0x30u) << 12) | ((x & 0xC0u) << 18);
            o[q] = __builtin_amdgcn_perm(0u, 0x54474341u, sel);  // "ACGT"
        }
        const uint64_t b = u << 4;
        if (b >= blo && b + 16 <= bhi) {
            *reinterpret_cast<uint4 *>(out + b) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (b + j >= blo && b + j < bhi) out[b + j] = (uint8_t)(o[j >> 2] >> (8 * (j & 3)));
        }
    }
}

// the exception bytes [elo, ehi) (not A/C/G/T in the original reads) back into the ASCII
__global__ void __launch_bounds__(256) k_patch(const uint64_t *__restrict__ pos, const uint8_t *__restrict__ byte,
                                               uint64_t elo, uint64_t ehi, uint8_t *__restrict__ out) {
    for (uint64_t i = elo + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ehi;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[pos[i]] = byte[i];
}

// offsets of reads of one length L: off[i] = i L
__global__ void __launch_bounds__(256) k_iota_off(uint64_t *off, uint64_t n1, uint64_t L) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n1; i += (uint64_t)gridDim.x * blockDim.x)
        off[i] = i * L;
}

}  // namespace ec
