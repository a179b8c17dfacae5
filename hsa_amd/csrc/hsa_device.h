// hsa_device.h -- device-side building blocks shared by the HIP sources.
//
// Rank layout (one per BWT direction): 64-byte blocks, block b covering the
// characters [192b, 192b+192) of the $-less BWT code string:
//   dwords 0..3  : Occ(A,C,G,T) over [0, 192b+96)          (uint4 h, mid-block)
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

// Occ over one block at in-block offset r (0..191).  The block's counts are at
// its MIDDLE (character 96, padding past the text counted as 'A' exactly as the
// reference's own samples do), so only the half holding r is fetched and decoded:
// 16 bytes of counts + 24 bytes of codes, at most six code words, forwards
// (r >= 96) or backwards (r < 96).
__device__ __forceinline__ void hsa_occ_in_block(const uint4 *__restrict__ q, uint32_t r, uint32_t o[4])
{
    const bool up = r >= 96u;
    const uint32_t *base = reinterpret_cast<const uint32_t *>(q);
    const uint4 h = q[0];
    const uint4 w4 = *reinterpret_cast<const uint4 *>(base + (up ? 12 : 4));   // words 8-11 | 0-3
    const uint2 w2 = *reinterpret_cast<const uint2 *>(base + (up ? 10 : 8));   // words 6-7  | 4-5
    const uint32_t w[6] = {up ? w2.x : w4.x, up ? w2.y : w4.y, up ? w4.x : w4.z,
                           up ? w4.y : w4.w, up ? w4.z : w2.x, up ? w4.w : w2.y};
    const uint32_t n = up ? r - 96u : r;               // prefix length inside the half
    const uint32_t qq = n >> 4;
    const uint32_t part = (n & 15u) ? ((1u << (2u * (n & 15u))) - 1u) : 0u;
    const uint32_t flip = up ? 0u : 0xffffffffu;        // lower half: count the suffix [n, 96)
    uint32_t n1 = 0, n2 = 0, n3 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) {
        const uint32_t pm = k < qq ? 0xffffffffu : (k == qq ? part : 0u);
        const uint32_t v = w[k] & (pm ^ flip);
        const uint32_t lo = v & 0x55555555u, hi = (v >> 1) & 0x55555555u;
        n3 += __popc(lo & hi);
        n1 += __popc(lo);
        n2 += __popc(hi);
    }
    n1 -= n3;
    n2 -= n3;
    const uint32_t cnt = up ? n : 96u - n;
    const uint32_t a = cnt - n1 - n2 - n3;
    if (up) { o[0] = h.x + a; o[1] = h.y + n1; o[2] = h.z + n2; o[3] = h.w + n3; }
    else    { o[0] = h.x - a; o[1] = h.y - n1; o[2] = h.z - n2; o[3] = h.w - n3; }
}

// Occ(p1, *) and Occ(p2, *) on one BWT: the two rank queries of one
// bidirectional step.  Returns the number of distinct 64-byte blocks (1 or 2).
__device__ __forceinline__ uint32_t hsa_occ_pair(const RankDir d, uint32_t p1, uint32_t p2,
                                                 uint32_t a[4], uint32_t b[4])
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    const uint32_t b1 = p1 / HSA_BLK_CHARS, b2 = p2 / HSA_BLK_CHARS;
    hsa_occ_in_block(d.blk + (size_t)b1 * 4, p1 - b1 * HSA_BLK_CHARS, a);
    hsa_occ_in_block(d.blk + (size_t)b2 * 4, p2 - b2 * HSA_BLK_CHARS, b);
    return 1u + (b2 != b1);
}

__device__ __forceinline__ void hsa_occ4(const RankDir d, uint32_t p, uint32_t o[4])
{
    p -= (p > d.isa0);
    const uint32_t bb = p / HSA_BLK_CHARS;
    hsa_occ_in_block(d.blk + (size_t)bb * 4, p - bb * HSA_BLK_CHARS, o);
}

// Occ of ONE character c over one block at in-block offset r (0..191): the width
// (bwt_cal_width, BWTSARangeForeward) and exact-tail steps need a single count.
// A code equal to c becomes 11 after XOR with the complement pattern of c, so one
// popcount per code word instead of three.
__device__ __forceinline__ uint32_t hsa_occ1_in_block(const uint4 *__restrict__ q, uint32_t r, uint32_t c)
{
    const bool up = r >= 96u;
    const uint32_t *base = reinterpret_cast<const uint32_t *>(q);
    const uint4 h = q[0];
    const uint4 w4 = *reinterpret_cast<const uint4 *>(base + (up ? 12 : 4));
    const uint2 w2 = *reinterpret_cast<const uint2 *>(base + (up ? 10 : 8));
    const uint32_t w[6] = {up ? w2.x : w4.x, up ? w2.y : w4.y, up ? w4.x : w4.z,
                           up ? w4.y : w4.w, up ? w4.z : w2.x, up ? w4.w : w2.y};
    const uint32_t n = up ? r - 96u : r;
    const uint32_t qq = n >> 4;
    const uint32_t part = (n & 15u) ? ((1u << (2u * (n & 15u))) - 1u) : 0u;
    const uint32_t flip = up ? 0u : 0xffffffffu;
    const uint32_t pat = ~(c * 0x55555555u);            // XOR turns code c into 0b11
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) {
        const uint32_t pm = k < qq ? 0xffffffffu : (k == qq ? part : 0u);
        const uint32_t x = w[k] ^ pat;
        cnt += __popc(x & (x >> 1) & (pm ^ flip) & 0x55555555u);
    }
    const uint32_t hc = c == 0 ? h.x : c == 1 ? h.y : c == 2 ? h.z : h.w;
    return up ? hc + cnt : hc - cnt;
}

// Occ(p1, c) and Occ(p2, c) on one BWT; returns the distinct 64-byte blocks (1 or 2).
__device__ __forceinline__ uint32_t hsa_occ1_pair(const RankDir d, uint32_t p1, uint32_t p2, uint32_t c,
                                                  uint32_t &a, uint32_t &b)
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    const uint32_t b1 = p1 / HSA_BLK_CHARS, b2 = p2 / HSA_BLK_CHARS;
    a = hsa_occ1_in_block(d.blk + (size_t)b1 * 4, p1 - b1 * HSA_BLK_CHARS, c);
    b = hsa_occ1_in_block(d.blk + (size_t)b2 * 4, p2 - b2 * HSA_BLK_CHARS, c);
    return 1u + (b2 != b1);
}
