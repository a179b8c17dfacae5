// hsa_device.h -- device-side building blocks shared by the HIP sources.
//
// Rank layout (one per BWT direction): 64-byte blocks, block b covering the
// characters [192b, 192b+192) of the $-less BWT code string:
//   dwords 0..3  : Occ(A,C,G,T) over [0, 192b)            (uint4 h)
//   dwords 4..15 : 192 two-bit codes, 16 per dword, LSB-first
// A rank query therefore touches exactly one 64-byte block.  The '$' skip of
// BWTOccValue (index -= index > inverseSa0, BWT.c:690) is applied before the
// lookup, which makes Occ(i, c) = #{p < i' : code[p] == c} -- the semantics the
// reference's sampled-Occ + SSE decode computes (BWT.c:682-837).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HSA_BLK_CHARS 192u

struct RankDir {
    const uint4 *blk;
    uint32_t isa0;
};

// Counts of C, G, T among the first r (0..192) codes of a block, plus A by
// complement: o = h + counts.
__device__ __forceinline__ void hsa_count_block(const uint4 h, const uint4 x, const uint4 y, const uint4 z,
                                                uint32_t r, uint32_t o[4])
{
    const uint32_t w[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w};
    uint32_t n1 = 0, n2 = 0, n3 = 0;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
        const int n = (int)r - 16 * q;
        const uint32_t m = n >= 16 ? 0xffffffffu : (n <= 0 ? 0u : ((1u << (2 * n)) - 1u));
        const uint32_t v = w[q] & m;
        const uint32_t lo = v & 0x55555555u, hi = (v >> 1) & 0x55555555u;
        n3 += __popc(lo & hi);
        n1 += __popc(lo);
        n2 += __popc(hi);
    }
    n1 -= n3;
    n2 -= n3;
    o[0] = h.x + r - n1 - n2 - n3;
    o[1] = h.y + n1;
    o[2] = h.z + n2;
    o[3] = h.w + n3;
}

// Occ(p1, *) and Occ(p2, *) on one BWT: the two rank queries of one
// bidirectional step.  Returns the number of 64-byte blocks fetched (1 or 2).
__device__ __forceinline__ uint32_t hsa_occ_pair(const RankDir d, uint32_t p1, uint32_t p2,
                                                 uint32_t a[4], uint32_t b[4])
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    const uint32_t b1 = p1 / HSA_BLK_CHARS, b2 = p2 / HSA_BLK_CHARS;
    const uint32_t r1 = p1 - b1 * HSA_BLK_CHARS, r2 = p2 - b2 * HSA_BLK_CHARS;
    const uint4 *q1 = d.blk + (size_t)b1 * 4;
    const uint4 *q2 = d.blk + (size_t)b2 * 4;
    const uint4 h1 = q1[0], x1 = q1[1], y1 = q1[2], z1 = q1[3];
    uint4 h2 = h1, x2 = x1, y2 = y1, z2 = z1;
    if (b2 != b1) {
        h2 = q2[0]; x2 = q2[1]; y2 = q2[2]; z2 = q2[3];
    }
    hsa_count_block(h1, x1, y1, z1, r1, a);
    hsa_count_block(h2, x2, y2, z2, r2, b);
    return 1u + (b2 != b1);
}

__device__ __forceinline__ void hsa_occ4(const RankDir d, uint32_t p, uint32_t o[4])
{
    p -= (p > d.isa0);
    const uint32_t bb = p / HSA_BLK_CHARS, r = p - bb * HSA_BLK_CHARS;
    const uint4 *q = d.blk + (size_t)bb * 4;
    hsa_count_block(q[0], q[1], q[2], q[3], r, o);
}
