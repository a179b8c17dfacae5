#pragma once
// hsa_trie.h -- the root tries: every string of up to D characters (D = the index's
// trie depth, HSA_TRIE_DEPTH, default 11) with the SA interval the rank steps would
// compute for it, so that a search path's first D steps are answered by one cached
// load each instead of a rank pair on two random 64-byte sectors of the multi-GB rank
// table.
//
// Why: every read's search starts at the root (the whole SA range) and every step of
// bwt_match_gap / bwt_match_exact / bwt_cal_width near the root works on a wide
// interval, whose two rank queries (k - 1, l) fall in different blocks.  In config 2
// about half of the search's steps extend a string of <= 11 characters (the
// one-substitution branches near the root; tools/exp/depth_hist.py).  All those
// strings together are a few tens of MB -- resident in the Infinity Cache -- where the
// rank table is 5.6 GB of uniformly random sectors.
//
// The intervals are the kernels' own arithmetic applied level by level (the builders
// below call the same occ_pair and the same formulas as k_search's expansion and
// k_widths' step), so a trie answer is bit-identical to the rank steps it replaces.
// The rank-query count stays the reference's: a step answered from a trie still
// counts its two queries (d_counters[2]); d_counters[10] counts the trie loads.
//
// Two tries, both with node p's children at 4 p + c on the next level:
//   search trie (k_search): c PREPENDED (backward search, BWTAllSARangesBackward_
//     Bidirection, 2BWT-Interface.c:235-272): entry {k, l, rev_k, L}, L = the
//     length of the string's shortest empty suffix (0: the string occurs), so an
//     exact tail that jumps several characters at once still counts the steps
//     bwt_match_exact takes before its interval empties (2BWT-Interface.c:375-381).
//     Plus one byte per node of levels 0..D-1: bit c = child 4p + c occurs.
//   width trie (k_widths): c APPENDED (forward extension on the reverse BWT,
//     BWTSARangeForeward, 2BWT-Interface.c:121-131): entry {k, l}.
// Level d (1..D) holds 4^d entries from entry (4^d - 4) / 3; the mask bytes of level
// d (0..D-1) start at byte (4^d - 1) / 3.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hsa_device.h"

#define HSA_TRIE_MAX_DEPTH 13u
#define HSA_TRIE_DEFAULT_DEPTH 12u

__host__ __device__ __forceinline__ uint64_t trie_base(uint32_t d) { return ((1ull << (2u * d)) - 4ull) / 3ull; }
__host__ __device__ __forceinline__ uint64_t trie_mbase(uint32_t d) { return ((1ull << (2u * d)) - 1ull) / 3ull; }

// search-trie entry: 32-bit intervals one uint4 {k, l, rk, L}; 64-bit two
// {k, l} {rk, L | 0}
template <typename IT> struct TrieC { IT v[4]; };   // the forward C table, by value

template <typename IT>
__device__ __forceinline__ void trie_s_load(const uint4 *t, uint64_t e, IT &k, IT &l, IT &rk, uint32_t &L)
{
    if constexpr (sizeof(IT) == 4) {
        const uint4 v = t[e];
        k = v.x; l = v.y; rk = v.z; L = v.w;
    } else {
        const uint4 u = t[2 * e], v = t[2 * e + 1];
        k = (uint64_t)u.x | (uint64_t)u.y << 32;
        l = (uint64_t)u.z | (uint64_t)u.w << 32;
        rk = (uint64_t)v.x | (uint64_t)v.y << 32;
        L = v.z;
    }
}

template <typename IT>
__device__ __forceinline__ void trie_s_store(uint4 *t, uint64_t e, IT k, IT l, IT rk, uint32_t L)
{
    if constexpr (sizeof(IT) == 4) {
        t[e] = make_uint4(k, l, rk, L);
    } else {
        t[2 * e] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)l, (uint32_t)(l >> 32));
        t[2 * e + 1] = make_uint4((uint32_t)rk, (uint32_t)(rk >> 32), L, 0u);
    }
}

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

// Level d -> level d + 1 of the search trie: one thread per node p of level d (the root
// for d = 0).  The children are the four intervals of the bidirectional step exactly
// as k_search's expansion computes them (2BWT-Interface.c:235-272).
//
// An interval past the text (l > T) can only come from an index whose two BWTs are not
// each other's reverse (test fixtures built from unrelated texts): the builders then
// raise *bad, store the string as absent (so no deeper level reads past the rank
// blocks), and the index keeps no trie.
template <typename IT, typename RD>
__global__ void __launch_bounds__(256) k_trie_search_level(RD fwd, IT T, TrieC<IT> Cg, uint32_t d,
                                                           uint4 *__restrict__ tr, uint8_t *__restrict__ mask,
                                                           unsigned *bad)
{
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= (1ull << (2u * d))) return;
    IT k = 0, l = T, rk = 0;
    uint32_t L = 0;
    if (d > 0) trie_s_load<IT>(tr, trie_base(d) + p, k, l, rk, L);
    const uint64_t ch = trie_base(d + 1) + 4 * p;
    uint32_t m = 0;
    if (k > l) {
        for (uint32_t c = 0; c < 4; ++c) trie_s_store<IT>(tr, ch + c, (IT)1, (IT)0, (IT)0, L);
    } else {
        IT oa[4], ob[4];
        const IT *const C = Cg.v;
        occ_pair(fwd, k, l + (IT)1, oa, ob);
        const IT erl = rk + (l - k);
        IT oc = 0;
        for (int c = 3; c >= 0; --c) {
            const IT dd = ob[c] - oa[c];
            const IT kc = C[c] + oa[c] + (IT)1, lc = C[c] + ob[c];
            const IT rkc = (erl - oc) - (lc - kc);
            oc += dd;
            bool ne = kc <= lc;
            if (ne && lc > T) { *bad = 1u; ne = false; }
            m |= (ne ? 1u : 0u) << c;
            if (ne) trie_s_store<IT>(tr, ch + c, kc, lc, rkc, 0u);
            else trie_s_store<IT>(tr, ch + c, kc <= lc ? (IT)1 : kc, kc <= lc ? (IT)0 : lc, rkc, d + 1u);
        }
    }
    mask[trie_mbase(d) + p] = (uint8_t)m;
}

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
