// hsa_device.h -- device-side building blocks shared by the HIP sources.
//
// Rank layout (one per BWT direction): one 16-byte block per 16 characters of the
// $-less BWT code string.  Block b (characters [16b, 16b + 16)) is one uint4:
//   x, y, z : Occ(A), Occ(C), Occ(G) over [0, 16b)
//   w       : the block's 16 two-bit codes, LSB-first (character 16b + j at bits 2j..2j+1)
// Occ(T) is implied: the four counts of a prefix sum to its length.  A rank query
// is therefore ONE 16-byte load and a popcount over the masked code word.
//
// Why so dense: on MI355X a wave-wide gather of 64 random lines costs the CU's
// texture pipeline (TA/TD) about two cycles per line and per load instruction, and
// the search kernel saturated it (TD busy 91 %) with the earlier 64-byte/192-char
// blocks, whose query took three load instructions on the same line.  The index
// grows to T bytes per direction (6 GB for an hg19-sized text, of 288 GB of HBM);
// HBM traffic stays one 64-byte sector per query.
//
// The '$' skip of BWTOccValue (index -= index > inverseSa0, BWT.c:690) is applied
// before the lookup, which makes Occ(i, c) = #{p < i' : code[p] == c} -- the
// semantics the reference's sampled-Occ + SSE decode computes (BWT.c:682-837).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HSA_BLK_CHARS 16u
#define HSA_SECTOR_BLOCKS 4u   // 16-byte blocks per 64-byte sector (statistics)

// v_c for a runtime base c in 0..3 as a select tree on the two bits of c.  The
// equality chain c == 0 ? v0 : c == 1 ? v1 : ... was compiled into nested divergent
// branches (an exec-mask save and restore per element) inside the search loops.
template <typename V>
__device__ __forceinline__ V hsa_sel4(uint32_t c, V v0, V v1, V v2, V v3)
{
#if HSA_PICK4_CHAIN                 // A/B builds only: the equality chain
    return c == 0 ? v0 : c == 1 ? v1 : c == 2 ? v2 : v3;
#else
    const bool b0 = (c & 1u) != 0;
    const V lo = b0 ? v1 : v0, hi = b0 ? v3 : v2;
    return (c & 2u) ? hi : lo;
#endif
}

struct RankDir {
    const uint4 *blk;
    uint32_t isa0;
};

#ifndef HSA_NT_RANK
#define HSA_NT_RANK 0
#endif
__device__ __forceinline__ uint4 hsa_blk_load(const uint4 *__restrict__ blk, uint32_t b)
{
#if HSA_NT_RANK
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(blk) + b);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return blk[b];
#endif
}

// Occ(p, A..T) of an already $-adjusted position p, from its block q.
__device__ __forceinline__ void hsa_occ4_q(const uint4 q, uint32_t p, uint32_t o[4])
{
    const uint32_t r = p & 15u;
    const uint32_t v = q.w & ((1u << (2u * r)) - 1u);        // r <= 15: shift <= 30
    const uint32_t lo = v & 0x55555555u, hi = (v >> 1) & 0x55555555u;
    const uint32_t n3 = __popc(lo & hi);
    const uint32_t n1 = __popc(lo) - n3, n2 = __popc(hi) - n3;
    o[0] = q.x + (r - n1 - n2 - n3);
    o[1] = q.y + n1;
    o[2] = q.z + n2;
    o[3] = p - o[0] - o[1] - o[2];
}

__device__ __forceinline__ void hsa_occ4_raw(const uint4 *__restrict__ blk, uint32_t p, uint32_t o[4])
{
    hsa_occ4_q(hsa_blk_load(blk, p >> 4), p, o);
}

// Occ(p, c) of an already $-adjusted position p from its block q: one popcount of the
// codes equal to c (XOR with the complement pattern of c turns them into 0b11).
__device__ __forceinline__ uint32_t hsa_occ1_q(const uint4 q, uint32_t p, uint32_t c)
{
    const uint32_t r = p & 15u;
    const uint32_t x = q.w ^ ~(c * 0x55555555u);
    const uint32_t n = __popc(x & (x >> 1) & 0x55555555u & ((1u << (2u * r)) - 1u));
    const uint32_t base = hsa_sel4(c, q.x, q.y, q.z, (p & ~15u) - q.x - q.y - q.z);
    return base + n;
}

// Occ(p1, *) and Occ(p2, *) on one BWT: the two rank queries of one bidirectional
// step.  Returns the number of distinct 64-byte sectors touched (1 or 2).
__device__ __forceinline__ uint32_t hsa_occ_pair(const RankDir d, uint32_t p1, uint32_t p2, uint32_t a[4], uint32_t b[4])
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    // a narrow interval has both ends in one block: then one load serves both.  The
    // second load is issued before the first is waited for (q2 is chosen after both):
    // with `q2 = q1; if (..) q2 = load` the compiler waits for q1 before the branch
    // and the two sectors of a wide interval cost two serial memory latencies.
    const uint32_t b1 = p1 >> 4, b2 = p2 >> 4;
    const bool two = b2 != b1;
    const uint4 q1 = hsa_blk_load(d.blk, b1);
    uint4 q2r = make_uint4(0, 0, 0, 0);
    if (two) q2r = hsa_blk_load(d.blk, b2);
    const uint4 q2 = two ? q2r : q1;
    hsa_occ4_q(q1, p1, a);
    hsa_occ4_q(q2, p2, b);
    return 1u + ((p1 >> 6) != (p2 >> 6));
}

__device__ __forceinline__ void hsa_occ4(const RankDir d, uint32_t p, uint32_t o[4])
{
    p -= (p > d.isa0);
    hsa_occ4_raw(d.blk, p, o);
}

// Occ(p1, c) and Occ(p2, c) on one BWT (width and exact steps); returns the distinct
// 64-byte sectors touched.
__device__ __forceinline__ uint32_t hsa_occ1_pair(const RankDir d, uint32_t p1, uint32_t p2, uint32_t c,
                                                  uint32_t &a, uint32_t &b)
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    const uint32_t b1 = p1 >> 4, b2 = p2 >> 4;    // both loads in flight (hsa_occ_pair)
    const bool two = b2 != b1;
    const uint4 q1 = hsa_blk_load(d.blk, b1);
    uint4 q2r = make_uint4(0, 0, 0, 0);
    if (two) q2r = hsa_blk_load(d.blk, b2);
    const uint4 q2 = two ? q2r : q1;
    a = hsa_occ1_q(q1, p1, c);
    b = hsa_occ1_q(q2, p2, c);
    return 1u + ((p1 >> 6) != (p2 >> 6));
}

// ---------------------------------------------------------------- 64-bit texts
// Texts of 2^32 characters or more (config 5; the reference's bwtint_t is 32-bit,
// 2BWT-Interface.h:26).  The blocks are the same 16-byte blocks, their counts kept
// modulo 2^32.  The high words come from the wrap table: a wrap of base c is the
// first block whose count of c reaches a multiple of 2^32 (there the block's low word
// drops below its predecessor's, since counts grow by <= 16 per block), so
//   Occ(16 b, c) = (wraps of c at blocks <= b) 2^32 + block b's low word.
// A text of i.i.d. bases passes 2^32 of one base only past ~17 Gbp, and a text under
// 2^36 characters has at most 15 wraps per base (HSA_MAX_WRAPS).  The table is the
// HSA_WRAP_HEAD bytes in front of block 0, read only when the index has a wrap at all
// (`any`, a uniform branch): an index without one pays nothing over the 32-bit rank,
// where a superblock table cost a cached load per rank query.
#define HSA_MAX_WRAPS 15u
#define HSA_WIDE_MAX_T (1ull << 36)
#define HSA_WRAP_HEAD 512u               // bytes allocated in front of every block array

struct RankDir64 {
    const uint4 *blk;
    uint64_t isa0;
    uint32_t any;                        // the index has a wrap
};

// the wrap table in front of block 0: [0] = the number of wraps, then (block, base) pairs by
// block from word 2
__device__ __host__ __forceinline__ const uint32_t *hsa_wrap_table(const uint4 *blk)
{
    return reinterpret_cast<const uint32_t *>(blk) - HSA_WRAP_HEAD / 4;
}

__device__ __forceinline__ void hsa_hi64(const uint32_t *__restrict__ wrap, uint32_t b, uint64_t o[3])
{
    // one loop over all wraps (<= 45), by block: entry j = (block, base) at [2j + 2]
    const uint32_t n = wrap[0];
#pragma unroll 1
    for (uint32_t j = 0; j < n; ++j) {
        const uint2 e = reinterpret_cast<const uint2 *>(wrap)[j + 1];
        if (b < e.x) break;
        const uint32_t c = e.y;
        o[0] += c == 0 ? 0x100000000ull : 0ull;
        o[1] += c == 1 ? 0x100000000ull : 0ull;
        o[2] += c == 2 ? 0x100000000ull : 0ull;
    }
}

__device__ __forceinline__ void hsa_occ4_q64(const uint4 q, const RankDir64 &d, uint64_t p, uint64_t o[4])
{
    const uint32_t r = (uint32_t)p & 15u;
    const uint32_t v = q.w & ((1u << (2u * r)) - 1u);
    const uint32_t lo = v & 0x55555555u, hi = (v >> 1) & 0x55555555u;
    const uint32_t n3 = __popc(lo & hi);
    const uint32_t n1 = __popc(lo) - n3, n2 = __popc(hi) - n3;
    o[0] = (uint64_t)q.x + (r - n1 - n2 - n3);
    o[1] = (uint64_t)q.y + n1;
    o[2] = (uint64_t)q.z + n2;
    if (d.any) hsa_hi64(hsa_wrap_table(d.blk), (uint32_t)(p >> 4), o);   // uniform: no wraps, no work
    o[3] = p - o[0] - o[1] - o[2];
}

__device__ __forceinline__ uint64_t hsa_occ1_q64(const uint4 q, const RankDir64 &d, uint64_t p, uint32_t c)
{
    uint64_t o[4];
    hsa_occ4_q64(q, d, p, o);
    return hsa_sel4(c, o[0], o[1], o[2], o[3]);
}

// The same interface as the 32-bit rank functions (k_search / k_widths are templated
// on the interval type and call these by overload).
__device__ __forceinline__ uint32_t occ_pair(const RankDir &d, uint32_t p1, uint32_t p2, uint32_t a[4], uint32_t b[4])
{
    return hsa_occ_pair(d, p1, p2, a, b);
}

__device__ __forceinline__ uint32_t occ1_pair(const RankDir &d, uint32_t p1, uint32_t p2, uint32_t c, uint32_t &a,
                                              uint32_t &b)
{
    return hsa_occ1_pair(d, p1, p2, c, a, b);
}

__device__ __forceinline__ uint32_t occ_pair(const RankDir64 &d, uint64_t p1, uint64_t p2, uint64_t a[4],
                                             uint64_t b[4])
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    const uint64_t b1 = p1 >> 4, b2 = p2 >> 4;
    const bool two = b2 != b1;
    const uint4 q1 = d.blk[b1];
    uint4 q2r = make_uint4(0, 0, 0, 0);
    if (two) q2r = d.blk[b2];
    const uint4 q2 = two ? q2r : q1;
    hsa_occ4_q64(q1, d, p1, a);
    hsa_occ4_q64(q2, d, p2, b);
    return 1u + ((p1 >> 6) != (p2 >> 6));
}

__device__ __forceinline__ uint32_t occ1_pair(const RankDir64 &d, uint64_t p1, uint64_t p2, uint32_t c, uint64_t &a,
                                              uint64_t &b)
{
    p1 -= (p1 > d.isa0);
    p2 -= (p2 > d.isa0);
    const uint64_t b1 = p1 >> 4, b2 = p2 >> 4;
    const bool two = b2 != b1;
    const uint4 q1 = d.blk[b1];
    uint4 q2r = make_uint4(0, 0, 0, 0);
    if (two) q2r = d.blk[b2];
    const uint4 q2 = two ? q2r : q1;
    a = hsa_occ1_q64(q1, d, p1, c);
    b = hsa_occ1_q64(q2, d, p2, c);
    return 1u + ((p1 >> 6) != (p2 >> 6));
}
