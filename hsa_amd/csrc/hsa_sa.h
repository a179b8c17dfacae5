// hsa_sa.h -- SA index -> text position on the device, shared by
// k_sa_position (hsa_sa.hip) and the splice path's kernel (hsa_splice.hip).
//
// BWTSaValue (BWT.c:1195-1220) walks LF (BWTPsiMinusValue, BWT.c:1142-1162, via
// BWTOccValueOnSpot, BWT.c:924-959) until the SA index is a multiple of the sampling
// interval, then adds the steps to the sampled value; BWTRetrievePositionFromSAIndex
// (2BWT-Interface.c:329-361) then binary-searches the chromosome block table for
// (chrID, 1-based position).  Every LF step is one 16-byte rank-block load (the
// character before the position and its count come from the same block).
#pragma once
#include "hsa_device.h"

struct SaView {
    const uint4 *blk;              // forward rank blocks
    uint32_t isa0;
    uint32_t C[4];
    const uint32_t *sa;            // sampled values; sa[0] = -1 as BWTLoad leaves it (BWT.c:222)
    uint32_t interval;
    const uint32_t *blocks;        // n_blocks rows (chrID, blockStart, blockEnd, ori), HSP.h:41-46
    uint32_t n_blocks;
};

// BWTPsiMinusValue: the LF map of SA index `index` (index != inverseSa0).
__device__ __forceinline__ uint32_t hsa_psi_minus(const SaView &a, uint32_t index)
{
    uint32_t i = index + 1u;
    i -= (i > a.isa0);                         // BWTOccValueOnSpot: '$' is not encoded (BWT.c:949)
    const uint32_t p = i - 1u;                 // the BWT character before i ...
    const uint4 q = a.blk[p >> 4];
    const uint32_t r = p & 15u;
    const uint32_t c = (q.w >> (2u * r)) & 3u;
    const uint32_t x = q.w ^ ~(c * 0x55555555u);
    const uint32_t n = __popc(x & (x >> 1) & 0x55555555u & ((1u << (2u * r)) - 1u));
    const uint32_t base = hsa_sel4(c, q.x, q.y, q.z, (p & ~15u) - q.x - q.y - q.z);
    const uint32_t cc = hsa_sel4(c, a.C[0], a.C[1], a.C[2], a.C[3]);
    return cc + base + n + 1u;                 // ... and its count up to and including it
}

// BWTSaValue: the text position of SA index `index`.
__device__ __forceinline__ uint32_t hsa_sa_value(const SaView &a, uint32_t index)
{
    uint32_t skipped = 0;
    while (index % a.interval != 0) {
        ++skipped;
        index = index == a.isa0 ? 0u : hsa_psi_minus(a, index);
    }
    return a.sa[index / a.interval] + skipped;
}

// The block search of BWTRetrievePositionFromSAIndex (h starts at nblock; where the
// reference would read past the table -- m >= nblock -- it stops as "not found", see
// oracle/hsa_oracle.c).  Returns whether a block holds occ; sid / ori only then.
__device__ __forceinline__ bool hsa_sa_block(const SaView &a, uint32_t occ, uint32_t &sid, uint32_t &ori)
{
    uint32_t l = 0, h = a.n_blocks;
    while (l <= h) {
        const uint32_t m = (h + l) >> 1;
        if (m >= a.n_blocks) break;
        const uint32_t start = a.blocks[4 * m + 1];
        if (start > occ) { h = m - 1u; continue; }
        const uint32_t end = a.blocks[4 * m + 2];
        if (end < occ) { l = m + 1u; continue; }
        sid = a.blocks[4 * m];
        ori = occ - start + a.blocks[4 * m + 3] + 1u;
        return true;
    }
    return false;
}
