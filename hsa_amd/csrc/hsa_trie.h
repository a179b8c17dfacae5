#pragma once
// hsa_trie.h -- the root width trie: every string of up to D characters (D = the index's
// trie depth, HSA_TRIE_DEPTH, default 12) with the SA interval the rank steps would
// compute for it, so that a search path's first D steps are answered by one cached
// load each instead of a rank pair on two random 64-byte sectors of the multi-GB rank
// table.
//
// Why: every read's search starts at the root (the whole SA range) and every step of
// bwt_match_gap / bwt_match_exact / bwt_cal_width near the root works on a wide
// interval, whose two rank queries (k - 1, l) fall in different blocks.  In config 2
// 45 % of k_widths' steps extend a string of <= 11 characters since the chain's last
// reset (tools/exp/depth_hist.py).  All those
// strings together are a few tens of MB -- resident in the Infinity Cache -- where the
// rank table is 5.6 GB of uniformly random sectors.
//
// The intervals are the kernel's own arithmetic applied level by level (the builder
// below calls the same occ_pair and the same formulas as k_widths' step), so a trie
// answer is bit-identical to the rank steps it replaces.
// The rank-query count stays the reference's: a step answered from a trie still
// counts its two queries (d_counters[2]); d_counters[10] counts the trie loads.
//
// The width trie (k_widths): c APPENDED (forward extension on the reverse BWT,
// BWTSARangeForeward, 2BWT-Interface.c:121-131): entry {k, l}; node p's children at
// 4 p + c on the next level.  Level d (1..D) holds 4^d entries from entry (4^d - 4) / 3.
// (A search trie for k_search -- c prepended, with exact-tail jumps -- was built and
// measured slower than the rank steps it replaced, at every depth, in large and in
// 100 000-read batches: DESIGN.md.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hsa_device.h"

#define HSA_TRIE_MAX_DEPTH 15u      // node numbers of a level stay below 2^32 (uint32_t)
#define HSA_TRIE_DEFAULT_DEPTH 12u

__host__ __device__ __forceinline__ uint64_t trie_base(uint32_t d) { return ((1ull << (2u * d)) - 4ull) / 3ull; }
template <typename IT> struct TrieC { IT v[4]; };   // the forward C table, by value

// width-trie entry: {k, l} of the reverse BWT
template <typename IT>
__device__ __forceinline__ void trie_w_load(const void *t, uint64_t e, IT &k, IT &l)
{
    if constexpr (sizeof(IT) == 4) {
        const uint2 v = reinterpret_cast<const uint2 *>(t)[e];
        k = v.x; l = v.y;
    } else {
        const uint4 v = reinterpret_cast<const uint4 *>(t)[e];
        k = (uint64_t)v.x | (uint64_t)v.y << 32;
        l = (uint64_t)v.z | (uint64_t)v.w << 32;
    }
}

template <typename IT>
__device__ __forceinline__ void trie_w_store(void *t, uint64_t e, IT k, IT l)
{
    if constexpr (sizeof(IT) == 4) reinterpret_cast<uint2 *>(t)[e] = make_uint2(k, l);
    else reinterpret_cast<uint4 *>(t)[e] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)l, (uint32_t)(l >> 32));
}

// An interval past the text (l > T) can only come from an index whose two BWTs are not
// each other's reverse (test fixtures built from unrelated texts): the builder then
// raises *bad, stores the string as absent (so no deeper level reads past the rank
// blocks), and the index keeps no trie.
// Level d -> level d + 1 of the width trie: the forward extension of k_widths' step
// (reverse BWT, forward C table; bwtaln.c:84-97).
template <typename IT, typename RD>
__global__ void __launch_bounds__(256) k_trie_width_level(RD rev, IT T, TrieC<IT> Cg, uint32_t d,
                                                          void *__restrict__ tw, unsigned *bad)
{
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= (1ull << (2u * d))) return;
    IT k = 0, l = T;
    if (d > 0) trie_w_load<IT>(tw, trie_base(d) + p, k, l);
    const uint64_t ch = trie_base(d + 1) + 4 * p;
    if (k > l) {
        for (uint32_t c = 0; c < 4; ++c) trie_w_store<IT>(tw, ch + c, (IT)1, (IT)0);
    } else {
        IT oa[4], ob[4];
        occ_pair(rev, k, l + (IT)1, oa, ob);
        for (uint32_t c = 0; c < 4; ++c) {
            IT kc = Cg.v[c] + oa[c] + (IT)1, lc = Cg.v[c] + ob[c];
            if (kc <= lc && lc > T) { *bad = 1u; kc = 1; lc = 0; }
            trie_w_store<IT>(tw, ch + c, kc, lc);
        }
    }
}
