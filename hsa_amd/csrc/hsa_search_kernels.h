#pragma once
// hsa_search_kernels.h -- the bwa_cal_sa_reg_gap per-read loop as two persistent kernels
// (templated on the interval type: 32-bit, the reference's bwtint_t, and 64-bit for
// texts of 2^32 characters or more), and the host helpers that plan and launch them.
// Included by hsa_search.hip (32-bit API) and hsa_search64.hip (64-bit API).
//
// k_widths: bwt_cal_width (bwtaln.c:73-98) for every (read, strand) of the batch --
//   the seed width and the whole-read width of the rc and the fwd strand, one work
//   item per lane, pulled from a global queue.  All lanes run the same short step
//   (one single-character rank pair on the reverse BWT), so the waves stay
//   converged.  Output: per (read, strand) a row of pruning bytes
//   min(bid,127) | (w[p] == w[p+1]) << 7 for the read and for the seed, and the
//   full w values (only gap_shadow reads them).
// k_search: per read, rc strand then fwd strand (bwtaln.c:343-359): copy the
//   strand's pruning bytes into LDS and run bwt_match_gap (bwtgap.c:118-331); the
//   first strand with hits wins; no hit on either -> HSA_F_FALLBACK (splice).
//
// One lane owns one read at a time (reads are pulled from a global queue with a
// wave-aggregated atomic, so a lane that finishes a cheap read immediately takes
// the next one: work-stealing at read granularity).  Every loop iteration of
// k_search performs at most ONE bidirectional rank step per lane (two Occ queries
// on the forward BWT, usually one 64-byte block), whatever the lane is doing --
// exact tail (bwt_match_exact) or expansion -- so all lanes issue their HBM loads
// together and the state machine in between is register/LDS work.  Control that
// needs no rank (pruned pops, hits) loops without touching the BWT.
//
// Per-lane state in LDS (160 KiB per CU): the pruning bytes of the current strand
// (everything bwt_match_gap's pruning reads: bwtgap.c:170, :256-263) and the
// stack's bucket heads.  Buckets are the REACHABLE scores only (a score table per
// regime maps aln_score -> dense bucket, order preserved), so `-n 4 -o 0` needs 6
// heads instead of the reference's 54 (bwtgap.c:18).  Stack entries (16 bytes + a
// 16-bit link) live in a per-lane pool in HBM; a bit mask in registers gives the
// lowest non-empty bucket (== gap_stack_t.best).  The child pushed LAST by an
// expansion is always the next pop when its bucket is the lowest, so it stays in
// registers ("virtual top").  A regime set without gap opens (max_gapo == 0: every
// entry stays in state M) runs a specialisation without the indel code.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "hsa_device.h"
#include "hsa_internal.h"
#include "hsa_trie.h"

#define MODE_GAPE 0x01
#define MODE_LOGGAP 0x04
#define MODE_NONSTOP 0x10
#define ST_M 0
#define ST_I 1
#define ST_D 2
#define NIL16 0xFFFFu
#define BLOCK 256
#define MAXB 128          // dense buckets per regime (BMask<2>)
#define MAXS 512          // score table length per regime (n_stacks <= MAXS)

enum : uint32_t { PH_IDLE = 0, PH_POP, PH_EXACT, PH_EXPAND, PH_EXIT, PH_END, PH_WAIT };

struct SearchArgs {
    RankDir fwd, rev;
    uint32_t T;
    uint32_t C[5];
    // 64-bit texts (IT = uint64_t kernels): the same, with superblock tables
    RankDir64 fwd64, rev64;
    uint64_t T64;
    uint64_t C64[5];
    const hsa_regime_t *regimes;
    const uint8_t *bmap;           // [2][MAXS]: aln_score -> dense bucket (0xFF: unreachable)
    uint32_t ntab;                 // score table entries per regime kept in LDS (>= every n_stacks, multiple of 8)
    const hsa_job_t *jobs;
    const int32_t *job_list;       // optional indirection (re-runs); null = identity
    int n_jobs;
    const uint8_t *codes;
    int32_t *n_aln;
    uint32_t *flags;
    uint64_t *hit_off;
    uint32_t *hits;
    uint64_t hit_cap;
    unsigned long long *ctr;       // [0] queue head [1] hit alloc [2] rank queries [3] blocks [4] pops [5] errors
                                   // [6] width item queue head
    const uint8_t *wb, *ws;        // width rows of k_widths (row = list position * 2 + strand),
    uint32_t *wg;                  //   64 rows interleaved; wg: full w values (gap_shadow only)
    uint32_t rb, rs, rg;           //   row capacities: bytes, bytes, words
    uint4 *pool;
    void *nxt;                     // pool links: uint16_t, or uint32_t in the huge pass
    uint32_t *hbuf;
    uint32_t pcap, hcap, nb;
    uint32_t off_heads, off_wb, off_ws;   // LDS byte offsets
    uint32_t nib_wb, nib_ws;              // 4-bit layout: LDS words per lane of the read / seed row
    uint32_t mm_buckets;           // 1: the bucket of every score is its n_mm (no gap opens, s_mm > 0)
    // device-side overflow re-run: the main pass appends reads that exceeded their
    // lane's capacity to ovf_list (count in ctr[8]); the re-run pass takes its read
    // count from n_dev and its queue head from ctr[qctr]
    int32_t *ovf_list;
    const unsigned long long *n_dev;
    uint32_t qctr;
    uint32_t ovf_ctr;              // counter that numbers this pass's ovf_list entries
    // caller-width mode (hsa_match_gap_batch, bwt_match_gap called directly): per job
    // strand and width_seed kind; k_widths_import builds the rows from the caller's
    // bwt_width_t pairs (cw), the search takes that one strand, and gap_shadow keeps
    // the full bid values (wbid) so the mutated widths can be handed back
    const hsa_mg_job_t *mg;
    int32_t *cw;
    int32_t *wbid;
    uint32_t *wq;                  // k_widths: rank queries of each forward-strand width row
    uint32_t batch_k;              // rare-event batching: at most this many lanes wait (see (A) in k_search)
    uint32_t batch_idle;           //   ... or run once the waiting lanes have idled this many lane-iterations
    // strand-split mode (small batches): work item p searches ONE strand of list position
    // p >> 1 (p even: rc, odd: fwd) on its own lane, so a read's two searches run side by
    // side instead of one after the other; k_split_finalize keeps the fwd strand only
    // when rc has no hit (bwtaln.c:343-359) and counts its work only then
    uint32_t split;
    int32_t *sp_n;                 // per item: hits, or -1 for a capacity overflow
    uint64_t *sp_off;
    uint32_t *sp_q, *sp_p;         //   its rank queries and pops (counted by the finalize)
    // the root width trie (hsa_trie.h) of the index, ktd levels (0: none, or not of this
    // instantiation's interval width): k_widths answers the steps of strings up to ktd
    // characters from ktw
    const void *ktw;
    uint32_t ktd;
    // cost order (main pass of a batch larger than the chip): k_widths writes each row's
    // final bid (wkey), k_order_* sort the list positions by it, most differences first,
    // and k_search takes its reads in that order (perm), so the costly searches do not
    // start last and set the launch's tail
    uint8_t *wkey;
    const int32_t *perm;
    uint32_t okey;                  // cost key with the tail length (default; HSA_ORDER_KEY=0: bid only)
    // lazy forward rows (k_widths_reads): a read whose rc search found nothing and whose
    // forward row was not computed goes to fwd_list (count *fwd_n); the forward pass
    // (fwd_only) searches just that strand
    int32_t *fwd_list;
    unsigned long long *fwd_n;
    uint32_t fwd_only;
    // lazy main pass: rows in two planes, the rc row of list position q at row q and its
    // forward row (when computed) at row rmap[q], so every width lane stores coalesced;
    // null: row q * 2 + strand
    int32_t *rmap;
    // strand-split tails (helpers, k_search): a strand search with no hit yet that has run
    // fr_budget pops while more lanes wait for work than the shared frontier holds offers
    // its live entries there; waiting lanes search them (each entry a sub-search rooted at
    // it) and report only whether the item has a hit.  The owner keeps searching in the
    // reference's order; when every sub-search of its frontier ended without a hit it stops
    // with no hits, which is its own search's answer: before a hit, a strand search expands
    // the same entries in any order ("Helpers").  fr_budget 0: off.
    uint32_t fr_budget, fr_demand, fr_cap;
    uint32_t *fr_ent;              // published chunks: FR_CH entries of FR_EW words each
    uint32_t *fr_tag;              // per chunk: entries << 26 | (item + 1)
    uint32_t *fr_rq;               // ready queue: chunk + 1 once the chunk is complete (0 before)
    uint32_t *fr_st;               // per item: chunks not yet searched | FR_DONE | FR_HIT
    unsigned long long *fr_q, *fr_p;   // per item: its sub-searches' rank queries and pops
    unsigned long long *fr_c;      // [0] chunks reserved [1] ready-queue head (taken) [2] items finished
                                   // [3] lanes waiting [4] offers [5] offers refused (capacity) [6] sub-
                                   // searches ended [7] owners answered by their helpers [8] sub-searches'
                                   // rank queries [9] ready-queue tail
};
#define FR_HIT 0x80000000u
#define FR_DONE 0x40000000u
#define FR_EW 8u                   // words per published entry (32- and 64-bit intervals)
#define FR_CH 16u                  // entries per chunk: one sub-search searches a chunk's sub-trees
#define FR_WALK 1024u              // largest stack a strand offers (the walk is a chain of dependent loads)
#ifndef HSA_HELPERS
#define HSA_HELPERS 1              // A/B builds: -DHSA_HELPERS=0 compiles the helpers out of k_search
#endif

// The kernel's arguments re-read from the kernarg segment where a rare path uses them
// (strand start and end, next read, hit staging): the asm barrier keeps the compiler
// from hoisting those loads out of the search loop, where holding every argument in
// SGPRs across the loop forced SGPR spills (v_writelane / v_readlane round trips).
typedef const __attribute__((address_space(4))) SearchArgs *ColdArgs;
__device__ __forceinline__ ColdArgs cold_args()
{
    ColdArgs p = (ColdArgs)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(p));
    return p;
}

// entry meta word: i:10 | state:2 | is_diff:1 | n_mm:7 | n_gapo:4 | n_gape:8
__device__ __forceinline__ uint32_t meta_pack(uint32_t i, uint32_t st, uint32_t isd, uint32_t mm, uint32_t go,
                                              uint32_t ge)
{
    return i | st << 10 | isd << 12 | mm << 13 | go << 20 | ge << 24;
}
#define M_I(m) ((int)((m) & 1023u))
#define M_ST(m) ((int)(((m) >> 10) & 3u))
#define M_ISD(m) ((int)(((m) >> 12) & 1u))
#define M_MM(m) ((int)(((m) >> 13) & 127u))
#define M_GO(m) ((int)(((m) >> 20) & 15u))
#define M_GE(m) ((int)((m) >> 24))

// control word: ph:3 | strand:1 | has_seed:1 | reg:1 | has_vt:1 | seed_alias:1 | ovf:2 | len:10 | seed_len:10
#define C_PH(c) ((c) & 7u)
#define C_STRAND(c) (((c) >> 3) & 1u)
#define C_SEED(c) (((c) >> 4) & 1u)
#define C_REG(c) (((c) >> 5) & 1u)
#define C_VT(c) (((c) >> 6) & 1u)
#define C_ALIAS(c) (((c) >> 7) & 1u)
#define C_OVF(c) (((c) >> 8) & 3u)
#define C_LEN(c) ((int)(((c) >> 10) & 1023u))
#define C_SLEN(c) ((int)(((c) >> 20) & 1023u))
#define SET_PH(c, p) ((c) = ((c) & ~7u) | (p))

// v[c] for a runtime c in 0..3 as selects (hsa_sel4): a dynamically indexed register
// array would be lowered through the private segment (scratch) of the dispatch.  The
// elements are passed by value at constant indices (a select between two element
// references became a dynamically indexed load).
template <typename V>
__device__ __forceinline__ V pick4(const V v[4], uint32_t c)
{
    return hsa_sel4<V>(c, v[0], v[1], v[2], v[3]);
}

// The interval type of a kernel instantiation: uint32_t (the reference's bwtint_t,
// 2BWT-Interface.h:26) or uint64_t (texts of 2^32 characters or more).
template <typename IT> struct Ix;
template <> struct Ix<uint32_t> {
    __device__ static const RankDir &fwd(const SearchArgs &a) { return a.fwd; }
    __device__ static const RankDir &rev(const SearchArgs &a) { return a.rev; }
    __device__ static uint32_t T(const SearchArgs &a) { return a.T; }
    __device__ static const uint32_t *C(const SearchArgs &a) { return a.C; }
};
template <> struct Ix<uint64_t> {
    __device__ static const RankDir64 &fwd(const SearchArgs &a) { return a.fwd64; }
    __device__ static const RankDir64 &rev(const SearchArgs &a) { return a.rev64; }
    __device__ static uint64_t T(const SearchArgs &a) { return a.T64; }
    __device__ static const uint64_t *C(const SearchArgs &a) { return a.C64; }
};

// A stack entry (gap_entry_t, bwtaln.h:52-58): k, l, rev_k and the meta word
// (rev_l = rev_k + (l - k)).  32-bit: one uint4 in the pool; 64-bit: two.
template <typename IT> struct Ent {
    IT x, y, z;
    uint32_t w;
};
#ifndef HSA_WAVES_SIMD
#define HSA_WAVES_SIMD 4      // k_search's launch bound: waves per SIMD its VGPRs must allow
#endif
#ifndef HSA_POOL_CHUNK
#define HSA_POOL_CHUNK 1
#endif
// Slot s of a lane's pool.  Default: uint4 element base + s * 64 (32-bit entries) or the
// two elements base + s * 128 and base + s * 128 + 64 (64-bit entries); base (pool_base)
// is the lane's slot 0, computed once per launch.  HSA_POOL_CHUNK: 64-byte chunks of
// consecutive slots per lane (4 entries, or 2 of 64 bits), chunk q of lane l at
// (q * 64 + l) * 64 B in the wave's region, so an expansion's burst of pushes
// (consecutive slots) writes whole sectors; the links likewise, 32 per 64 B.  The wave's
// region is sized for pcap rounded up to 32 slots (the scratch reservation does so).
template <typename IT>
__device__ __forceinline__ size_t pool_base(size_t wv, uint32_t pcap, int lane)
{
#if HSA_POOL_CHUNK
    return (sizeof(IT) == 4 ? 1u : 2u) * wv * (size_t)((pcap + 31u) & ~31u) * 64 + (size_t)lane * 4;
#else
    return (sizeof(IT) == 4 ? 1u : 2u) * wv * pcap * 64 + (size_t)lane;
#endif
}
template <typename IT>
__device__ __forceinline__ size_t ent_at(size_t base, uint32_t slot)
{
#if HSA_POOL_CHUNK
    constexpr uint32_t EQ = sizeof(IT) == 4 ? 4u : 2u, U = sizeof(IT) == 4 ? 1u : 2u;
    return base + (size_t)(slot / EQ) * 256 + (slot % EQ) * U;
#else
    return base + (size_t)slot * (sizeof(IT) == 4 ? 64 : 128);
#endif
}
template <typename IT>
__device__ __forceinline__ Ent<IT> ent_load(const uint4 *pool, size_t base, uint32_t slot)
{
    const size_t i = ent_at<IT>(base, slot);
    if constexpr (sizeof(IT) == 4) {
        const uint4 v = pool[i];
        return Ent<IT>{v.x, v.y, v.z, v.w};
    } else {
        const uint4 u = pool[i], v = pool[i + (HSA_POOL_CHUNK ? 1 : 64)];
        return Ent<IT>{(uint64_t)u.x | (uint64_t)u.y << 32, (uint64_t)u.z | (uint64_t)u.w << 32,
                       (uint64_t)v.x | (uint64_t)v.y << 32, v.z};
    }
}
template <typename IT>
__device__ __forceinline__ void ent_store(uint4 *pool, size_t base, uint32_t slot, const Ent<IT> &e)
{
    const size_t i = ent_at<IT>(base, slot);
    if constexpr (sizeof(IT) == 4) {
        pool[i] = make_uint4(e.x, e.y, e.z, e.w);
    } else {
        pool[i] = make_uint4((uint32_t)e.x, (uint32_t)(e.x >> 32), (uint32_t)e.y, (uint32_t)(e.y >> 32));
        pool[i + (HSA_POOL_CHUNK ? 1 : 64)] = make_uint4((uint32_t)e.z, (uint32_t)(e.z >> 32), e.w, 0u);
    }
}
// staged words per hit (HB) and words per output hit record: bwt_aln1_t (bwtaln.h:41-50)
// for 32-bit intervals; hsa_aln64_t (include/hsa_gpu.h) for 64-bit ones
template <typename IT> struct HitW { static constexpr uint32_t STAGE = sizeof(IT) == 4 ? 9u : 10u;
                                     static constexpr uint32_t OUT = sizeof(IT) == 4 ? 9u : 14u; };

__device__ __forceinline__ int int_log2(uint32_t v)   // bwtgap.c:107-116
{
    int c = 0;
    if (v & 0xffff0000u) { v >>= 16; c |= 16; }
    if (v & 0xff00) { v >>= 8; c |= 8; }
    if (v & 0xf0) { v >>= 4; c |= 4; }
    if (v & 0xc) { v >>= 2; c |= 2; }
    if (v & 0x2) c |= 1;
    return c;
}

template <int MW> struct BMask;
template <> struct BMask<0> {        // <= 32 buckets: one 32-bit word
    uint32_t m0 = 0;
    __device__ __forceinline__ void clear() { m0 = 0; }
    __device__ __forceinline__ bool any() const { return m0 != 0; }
    __device__ __forceinline__ int lowest() const { return m0 ? __ffs(m0) - 1 : (1 << 30); }
    __device__ __forceinline__ bool test(int b) const { return (m0 >> b) & 1u; }
    __device__ __forceinline__ void set(int b) { m0 |= 1u << b; }
    __device__ __forceinline__ void reset(int b) { m0 &= ~(1u << b); }
};
template <> struct BMask<1> {
    uint64_t m0 = 0;
    __device__ __forceinline__ void clear() { m0 = 0; }
    __device__ __forceinline__ bool any() const { return m0 != 0; }
    __device__ __forceinline__ int lowest() const { return m0 ? __ffsll((unsigned long long)m0) - 1 : (1 << 30); }
    __device__ __forceinline__ bool test(int b) const { return (m0 >> b) & 1ull; }
    __device__ __forceinline__ void set(int b) { m0 |= 1ull << b; }
    __device__ __forceinline__ void reset(int b) { m0 &= ~(1ull << b); }
};
template <> struct BMask<2> {
    uint64_t m0 = 0, m1 = 0;
    __device__ __forceinline__ void clear() { m0 = m1 = 0; }
    __device__ __forceinline__ bool any() const { return (m0 | m1) != 0; }
    __device__ __forceinline__ int lowest() const
    {
        if (m0) return __ffsll((unsigned long long)m0) - 1;
        if (m1) return 64 + __ffsll((unsigned long long)m1) - 1;
        return 1 << 30;
    }
    __device__ __forceinline__ bool test(int b) const { return b < 64 ? ((m0 >> b) & 1ull) : ((m1 >> (b - 64)) & 1ull); }
    __device__ __forceinline__ void set(int b) { if (b < 64) m0 |= 1ull << b; else m1 |= 1ull << (b - 64); }
    __device__ __forceinline__ void reset(int b) { if (b < 64) m0 &= ~(1ull << b); else m1 &= ~(1ull << (b - 64)); }
};

// Pruning element of one read position, as k_widths writes it and k_search keeps it
// in LDS: min(bid, BIDM) | (w[p] == w[p+1]) << BIDB | (code & 3) << CSH |
// (code > 3) << (CSH + 2), code being the strand sequence's base at p.  A bid is
// only ever compared with m, m - 1 or m_seed - 1 (bwtgap.c:170, :256-263), all
// <= max(max_diff, max_seed_diff), so capping it at BIDM is exact while that bound
// is < BIDM: 8-bit elements (4-bit bid) for bounds <= 14, else 16-bit (8-bit bid).
// The base code keeps exactly what bwt_match_gap derives from it: c > 3 (N) and
// (c + j) & 3 (bwtgap.c:305-306).
template <typename WT> struct WFmt {
    static constexpr bool NIB = false;
    static constexpr uint32_t BIDB = sizeof(WT) == 1 ? 4u : 8u;
    static constexpr uint32_t BIDM = (1u << BIDB) - 1u;
    static constexpr uint32_t EQ = 1u << BIDB;
    static constexpr uint32_t CSH = BIDB + 1u;
    static constexpr uint32_t EB = 8u * sizeof(WT);           // bits per element
    static constexpr uint32_t EPW = 4u / sizeof(WT);          // elements per u32
    __device__ static uint32_t code_bits(uint32_t c) { return (c & 3u) << CSH | (c > 3 ? 4u : 0u) << CSH; }
    __device__ static uint32_t code(uint32_t v) { return (v >> CSH) & 7u; }   // 0..3, or 4..7 for N
};

// 4-bit elements for long reads (k_search only): min(bid, 7) | eq << 3, eight per LDS
// word, exact while max(max_diff, max_seed_diff) <= 6.  k_widths still writes the
// 8-bit rows to HBM; k_search packs them into LDS at each strand start and reads the
// base codes from the HBM row (L2-resident), so a 250 bp read needs 126 B of LDS per
// lane instead of 252 B and the CU holds twice the waves.
struct WNib { uint8_t v; };
template <> struct WFmt<WNib> {
    static constexpr bool NIB = true;
    static constexpr uint32_t BIDB = 3u, BIDM = 7u, EQ = 8u, EB = 4u, EPW = 8u;
};

// four 8-bit elements (WFmt<uint8_t>) -> four 4-bit ones in the low 16 bits
__device__ __forceinline__ uint32_t nib4(uint32_t x)
{
    uint32_t b = x & 0x0F0F0F0Fu;                                   // bids, <= 15 per byte
    const uint32_t ge7 = ((b + 0x09090909u) >> 4) & 0x01010101u;     // bid >= 7
    b = (b & ~(ge7 * 0x0Fu)) | ge7 * 7u;
    uint32_t n = b | ((x >> 4) & 0x01010101u) << 3;                   // | eq << 3
    n = (n | n >> 4) & 0x00FF00FFu;
    return (n | n >> 8) & 0xFFFFu;
}

#ifdef HSA_DIAG
// Diagnostic build only (-DHSA_DIAG, never the product library): per-workgroup
// start/end s_memtime and s_memrealtime of the last launch, for the in-kernel
// clock and the workgroup-duration spread.
static __device__ unsigned long long g_diag[8192 * 4];
// event counters: 0 width steps, 1 exact steps, 2 expand steps, 3 virtual-top pops,
// 4 pool pops, 5 outer iterations (per wave), 6 lanes stepping summed over outer
// iterations, 7 control-loop iterations (per wave), 8 entries flushed to the pool,
// 9..12 shader cycles per wave in acquisition / control / rank-load wait / apply,
// 13 gap_shadow calls with last_diff_pos > 0, 14 their summed last_diff_pos,
// 15 strand starts, 16/17 exact/expand steps on a unique interval (l == k), 18/19
// width steps on a unique interval / all width steps; maxima over the launch's reads
// (a read = acquisition to finish_job, both strands): 21 rank steps, 22 s_memrealtime
// ticks (100 MHz), 23 pops; 24 / 25 rank steps of the longest item that ended with /
// without hits (split mode: an item is one strand)
static __device__ unsigned long long g_dctr[32];
#define DC(i) (++dc[i])
#else
#define DC(i) ((void)0)
#endif

// ---------------------------------------------------------------- k_widths
// bwt_cal_width type 1 (bwtaln.c:84-97) of every (read, strand): the whole read
// (width_back) and its last seed_len bases (width_seed, bwtaln.c:344-348).  The
// strand-1 sequence is the reverse complement (seq_reverse(.., 1), bwtaln.c:337).
// Forward extension on the reverse BWT with the forward C table
// (BWTSARangeForeward, 2BWT-Interface.c:121-131).
//
// One lane per (read, strand) row, rows in order, so a wave's 64 rows are stored
// interleaved -- element e of row R at (R / 64 * cap + e) * 64 + R % 64 -- and every
// store of a step is one coalesced 256-byte wave store.  The two chains of a row
// (read and seed) are independent, so each iteration advances both: two rank pairs
// in flight per lane.  All reads of a batch have similar lengths, so the lanes stay
// converged without a work queue.
template <typename IT> struct WChain {
    IT k, l;
    uint32_t bid;
    IT prevw;
    uint32_t acc;
    uint32_t tl, tix;              // width trie: characters since the last reset, and their node
    uint32_t lr;                   // position of the last reset (the cost order's tail length)
};

template <typename WT, typename IT>
__device__ __forceinline__ void width_step(const SearchArgs &a, WChain<IT> &ch, uint32_t t, uint32_t n, uint32_t c,
                                           uint32_t cbits, uint32_t *__restrict__ brow, IT *__restrict__ wrow,
                                           uint32_t &st_q, uint32_t &st_b, uint32_t &st_t)
{
    using F = WFmt<WT>;
    IT w;
    if (t < n) {
        if (c < 4) {
            if (ch.tl < a.ktd) {
                // a string of <= ktd characters since the reset: its interval from the
                // width trie (the same forward extension, hsa_trie.h)
                ch.tix = ch.tix * 4u + c;
                ++ch.tl;
                trie_w_load<IT>(a.ktw, trie_base(ch.tl) + ch.tix, ch.k, ch.l);
                ++st_t;
            } else {
                IT ok, ol;
                st_b += occ1_pair(Ix<IT>::rev(a), ch.k, ch.l + 1u, c, ok, ol);
                const IT cc = pick4(Ix<IT>::C(a), c);
                ch.k = cc + ok + 1u;
                ch.l = cc + ol;
            }
            st_q += 2;
        }
        if (ch.k > ch.l || c > 3) { ch.k = 0; ch.l = Ix<IT>::T(a); ++ch.bid; ch.tl = 0; ch.tix = 0; ch.lr = t; }
        w = ch.l - ch.k + 1u;
    } else {
        w = 0; ++ch.bid;                                         // width[len] = {0, ++bid}
    }
    // element t-1 is final now (its eq bit needs w[t]); elements go out a word at a time
    if (t > 0) {
        if (ch.prevw == w) ch.acc |= F::EQ << (((t - 1) % F::EPW) * F::EB);
        if ((t - 1) % F::EPW == F::EPW - 1) { brow[((t - 1) / F::EPW) * 64] = ch.acc; ch.acc = 0; }
    }
    ch.acc |= ((ch.bid < F::BIDM ? ch.bid : F::BIDM) | cbits) << ((t % F::EPW) * F::EB);
    if (wrow) wrow[t * 64] = w;
    ch.prevw = w;
    if (t == n) brow[(t / F::EPW) * 64] = ch.acc;
}

// One width row: both chains (the whole strand sequence and its last seed_len bases) of
// list position q's strand; returns the rank queries, 64-byte sectors and trie loads it
// took, and the chain's final bid (width[len].bid = the bid of the last base + 1).
struct WRow { uint32_t q, b, t, bid, tail; };

// The cost key of a row (SearchArgs::wkey): its final bid, and with okey the length of
// its last segment (positions after the last reset, where the search starts with the
// least slack): a short one lets the search branch sooner.
__device__ __forceinline__ uint8_t cost_key(const SearchArgs &a, const WRow &w)
{
    const uint32_t b = w.bid < 15u ? w.bid : 15u;
    if (!a.okey) return (uint8_t)(w.bid < 255u ? w.bid : 255u);
    return (uint8_t)(b << 4 | (w.tail < 16u ? 2u : w.tail < 48u ? 1u : 0u));
}

template <typename WT, typename IT>
__device__ __forceinline__ WRow width_row(const SearchArgs &a, uint32_t R, uint32_t strand, const hsa_job_t &J)
{
    using F = WFmt<WT>;
    const uint32_t len = J.len;
    const uint64_t off = J.off;
    const bool has_seed = (int)len > J.seed_len;
    const uint32_t slen = has_seed ? (uint32_t)J.seed_len : 0u;
    const size_t rb = R >> 6, rl = R & 63u;
    uint32_t *const brow = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(a.wb)) + rb * (a.rb / 4) * 64 + rl;
    uint32_t *const srow = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(a.ws)) + rb * (a.rs / 4) * 64 + rl;
    IT *const wrow = reinterpret_cast<IT *>(a.wg) + rb * a.rg * 64 + rl;
    WChain<IT> f{0, Ix<IT>::T(a), 0, 0, 0, 0, 0}, sd{0, Ix<IT>::T(a), 0, 0, 0, 0, 0};
    uint32_t st_q = 0, st_b = 0, st_t = 0;
    const uint32_t s0 = len - slen;
#ifndef HSA_CODECACHE
#define HSA_CODECACHE 1                    // A/B builds: -DHSA_CODECACHE=0 loads a byte every step
#endif
    // Each chain walks its read one position per step (forwards, or backwards on the rc
    // strand), so the 4-byte word of its last base is kept in registers and a load goes
    // out every fourth step.  The codes buffer is 4-byte aligned and padded past its last
    // read (hsa_device_batch_t.d_codes), so the word load stays inside it.
    uint32_t cq[2] = {0xFFFFFFFFu, 0xFFFFFFFFu}, cword[2] = {0u, 0u};
    auto base = [&](uint32_t sp, int ch) -> uint32_t {
        const uint64_t ix = off + (strand ? len - 1u - sp : sp);
        uint32_t c;
        if constexpr (HSA_CODECACHE) {
            const uint32_t wq = (uint32_t)(ix >> 2);
            if (wq != cq[ch]) {
                cword[ch] = *reinterpret_cast<const uint32_t *>(a.codes + (ix & ~(uint64_t)3));
                cq[ch] = wq;
            }
            c = (cword[ch] >> (((uint32_t)ix & 3u) * 8u)) & 0xFFu;
        } else {
            c = a.codes[ix];
        }
        return strand && c < 4 ? 3u - c : c;
    };
    for (uint32_t t = 0; t <= len; ++t) {
        const uint32_t cf = t < len ? base(t, 0) : 4u;
        // the read's elements also carry the strand sequence's base (k_search's getc)
        width_step<WT, IT>(a, f, t, len, cf, t < len ? F::code_bits(cf) : 0u, brow, wrow, st_q, st_b, st_t);
        if (has_seed && t <= slen) {
            const uint32_t cs = t < slen ? base(s0 + t, 1) : 4u;
            width_step<WT, IT>(a, sd, t, slen, cs, 0u, srow, nullptr, st_q, st_b, st_t);
        }
    }
    return WRow{st_q, st_b, st_t, f.bid, len - f.lr};
}

// one atomic per wave and counter (the kernels' lanes all reach it)
__device__ __forceinline__ void wave_add(unsigned long long *c, unsigned long long v)
{
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(c, v);
}

#define HSA_NOFWD 0xFFFFFFFFu        // wq: this read's forward row was not computed
#define HSA_F_NEEDFWD 0x100u         // k_search internal: rc had no hit, forward row missing

// One lane per row (rows in order): row = list position * 2 + strand.  The forward
// strand's rows are computed speculatively and count as the reference's work only
// when k_search searches that strand (ctr[13]: all of them).
template <typename WT, typename IT = uint32_t>
__global__ void __launch_bounds__(BLOCK) k_widths(SearchArgs a)
{
    const uint32_t R = blockIdx.x * BLOCK + threadIdx.x;     // row = list position * 2 + strand
    const uint32_t n_jobs = a.n_dev ? (uint32_t)*a.n_dev : (uint32_t)a.n_jobs;
    const uint32_t q = R >> 1, strand = R & 1u;
    WRow w{0, 0, 0, 0};
    if (R < 2u * n_jobs) {
        const hsa_job_t J = a.jobs[a.job_list ? a.job_list[q] : (int)q];
        w = width_row<WT, IT>(a, R, strand, J);
        if (!strand) a.wq[q] = w.q;
        if (a.wkey) a.wkey[R] = cost_key(a, w);
    }
    // rank queries: the reverse-complement strand is always searched (bwtaln.c:343)
    wave_add(&a.ctr[2], strand ? w.q : 0u);
    wave_add(&a.ctr[7], strand ? w.q : 0u);
    wave_add(&a.ctr[13], strand ? 0u : w.q);
    wave_add(&a.ctr[3], w.b);
    wave_add(&a.ctr[10], w.t);
}

// One lane per read, one strand's row each.
// mode 1 (main pass of a large batch): the rc row of every read; a read whose rc search
//   cannot have a hit -- its root is pruned when the last base's bid exceeds max_diff
//   (bwtgap.c:170) -- goes to list2 for its forward row; the others get wq = HSA_NOFWD
//   and k_search hands them to the forward pass if rc finds nothing (bwtaln.c:343-359).
// mode 3: the forward rows of list2 (the speculative count, as k_widths').
// mode 2 (the forward pass): the forward rows of the reads k_search listed, the
//   reference's work.
template <typename WT, typename IT = uint32_t>
__global__ void __launch_bounds__(BLOCK) k_widths_reads(SearchArgs a, uint32_t mode, int32_t *list2,
                                                        unsigned long long *n2)
{
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t n_jobs = mode == 3 ? (uint32_t)*n2 : a.n_dev ? (uint32_t)*a.n_dev : (uint32_t)a.n_jobs;
    WRow w{0, 0, 0, 0};
    bool more = false;
    if (p < n_jobs) {
        const uint32_t q = mode == 3 ? (uint32_t)list2[p] : p;
        const hsa_job_t J = a.jobs[a.job_list ? a.job_list[q] : (int)q];
        // mode 1: the rc plane (row q); mode 3: the forward plane after it (row n_al + p);
        // mode 2 (forward pass, no plane map): row 2 p
        const uint32_t R = mode == 1 ? q : mode == 3 ? (uint32_t)(((uint32_t)a.n_jobs + 63u) & ~63u) + p : 2u * q;
        w = width_row<WT, IT>(a, R, mode == 1 ? 1u : 0u, J);
        if (mode == 3) a.rmap[q] = (int32_t)R;
        const uint8_t key = cost_key(a, w);
        if (mode == 1) {
            more = (int)w.bid - 1 > J.max_diff;
            a.wq[q] = HSA_NOFWD;
            if (a.wkey) { a.wkey[2 * q + 1] = key; a.wkey[2 * q] = 255u; }
        } else if (mode == 3) {
            a.wq[q] = w.q;
            if (a.wkey) a.wkey[2 * q] = key;
        }
    }
    if (mode == 1) {                                    // list2: one atomic per wave
        const uint64_t m = __ballot(more);
        const int lane = (int)(threadIdx.x & 63);
        unsigned long long b = 0;
        if (m && lane == __ffsll((unsigned long long)m) - 1) b = atomicAdd(n2, (unsigned long long)__popcll(m));
        b = __shfl(b, __ffsll((unsigned long long)(m ? m : 1ull)) - 1);
        if (more) list2[b + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)p;
    }
    const uint32_t rq = mode == 1 ? w.q : 0u, fq = mode == 2 ? w.q : 0u, sq = mode == 3 ? w.q : 0u;
    wave_add(&a.ctr[2], rq + fq);
    wave_add(&a.ctr[7], rq + fq);
    wave_add(&a.ctr[13], fq + sq);
    wave_add(&a.ctr[14], fq);
    wave_add(&a.ctr[3], w.b);
    wave_add(&a.ctr[10], w.t);
}

// Caller-width mode: the width rows of each call from the caller's bwt_width_t pairs
// (hsa_match_gap_batch) -- the same element format and row layout k_widths writes;
// the row of list position q is q * 2 + strand.  Besides the pruning elements and the
// full w values, the full bids go to wbid: gap_shadow rewrites them (bwtgap.c:101).
template <typename WT>
__global__ void __launch_bounds__(BLOCK) k_widths_import(SearchArgs a)
{
    using F = WFmt<WT>;
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t n_jobs = a.n_dev ? (uint32_t)*a.n_dev : (uint32_t)a.n_jobs;
    if (q >= n_jobs) return;
    const int job = a.job_list ? a.job_list[q] : (int)q;
    const hsa_job_t J = a.jobs[job];
    const hsa_mg_job_t M = a.mg[job];
    const uint32_t R = q * 2u + (uint32_t)(M.strand & 1);
    const size_t rb = R >> 6, rl = R & 63u;
    uint32_t *const brow = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(a.wb)) + rb * (a.rb / 4) * 64 + rl;
    uint32_t *const srow = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(a.ws)) + rb * (a.rs / 4) * 64 + rl;
    uint32_t *const wrow = a.wg + rb * a.rg * 64 + rl;
    int32_t *const drow = a.wbid + rb * a.rg * 64 + rl;
    // elements 0..n of one row; element t: min(bid, BIDM) | (w[t] == w[t+1]) | base code.
    // A prefix row (HSA_MG_PREFIX: the first n entries of a longer bwt_cal_width row, the
    // splice seeds' widths, bwtgap.c:807) has the terminal {0, bid of entry n - 1, + 1}.
    const bool prefix = M.seed == HSA_SEED_ALIAS && M.ws_off == HSA_MG_PREFIX;
    auto emit = [&](uint32_t *row, const int32_t *w, uint32_t n, bool read_row) {
        uint32_t acc = 0;
        uint32_t wt = (uint32_t)w[0];
        for (uint32_t t = 0; t <= n; ++t) {
            const uint32_t bid = prefix && t == n ? (n ? (uint32_t)w[2 * t - 1] + 1u : 1u) : (uint32_t)w[2 * t + 1];
            const uint32_t wn = t + 1 < n || (t + 1 == n && !prefix) ? (uint32_t)w[2 * t + 2] : 0u;
            uint32_t e = bid < F::BIDM ? bid : F::BIDM;
            if (t < n && wt == wn) e |= F::EQ;
            if (read_row && t < n) e |= F::code_bits(a.codes[J.off + t]);
            acc |= e << ((t % F::EPW) * F::EB);
            if (t % F::EPW == F::EPW - 1 || t == n) { row[(t / F::EPW) * 64] = acc; acc = 0; }
            if (read_row) { wrow[t * 64] = wt; drow[t * 64] = (int32_t)bid; }
            wt = wn;
        }
    };
    emit(brow, a.cw + 2 * M.wb_off, J.len, true);
    if (M.seed == HSA_SEED_OWN) emit(srow, a.cw + 2 * M.ws_off, (uint32_t)J.seed_len, false);
}

// Caller-width mode: width_back after the search (gap_shadow rewrote it in the rows)
// back into the caller's pairs.  Reads that overflowed this pass are skipped: the
// re-run that completes them exports them.
static __global__ void __launch_bounds__(BLOCK) k_widths_export(SearchArgs a)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t n_jobs = a.n_dev ? (uint32_t)*a.n_dev : (uint32_t)a.n_jobs;
    if (q >= n_jobs) return;
    const int job = a.job_list ? a.job_list[q] : (int)q;
    if (a.flags[job] & HSA_F_OVERFLOW) return;
    const hsa_job_t J = a.jobs[job];
    const hsa_mg_job_t M = a.mg[job];
    if (M.seed == HSA_SEED_ALIAS && M.ws_off == HSA_MG_PREFIX) return;   // a row's prefix, read only
    const uint32_t R = q * 2u + (uint32_t)(M.strand & 1);
    const size_t base = (R >> 6) * (size_t)a.rg * 64 + (R & 63u);
    int32_t *const o = a.cw + 2 * M.wb_off;
    for (uint32_t t = 0; t <= J.len; ++t) {
        o[2 * t] = (int32_t)a.wg[base + t * 64];
        o[2 * t + 1] = a.wbid[base + t * 64];
    }
}


// Cost order of a batch's reads (see SearchArgs::wkey): the lower bid of a read's two
// strands -- a lower bound on the differences of its best strand (bwtaln.c:84-97) --
// bucketed into 16 bins, most differences first; order within a bin is arbitrary (every
// read's result is independent of when it is searched).
__device__ __forceinline__ uint32_t order_bin(const SearchArgs &a, uint32_t q)
{
    const uint32_t k0 = a.wkey[2 * q], k1 = a.wkey[2 * q + 1];
    const uint32_t k = k0 < k1 ? k0 : k1;
    if (a.okey) {                   // bid x 3 tail classes, costly first
        const uint32_t v = (k >> 4) * 3u + (k & 15u);
        return 15u - (v < 15u ? v : 15u);
    }
    return 15u - (k < 15u ? k : 15u);
}

static __global__ void __launch_bounds__(BLOCK) k_order_hist(SearchArgs a, uint32_t *hist)
{
    __shared__ uint32_t h[16];
    if (threadIdx.x < 16) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    if (q < (uint32_t)a.n_jobs) atomicAdd(&h[order_bin(a, q)], 1u);
    __syncthreads();
    if (threadIdx.x < 16 && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// hist[16] -> exclusive offsets in hist[16..31] (one thread)
static __global__ void k_order_scan(uint32_t *hist)
{
    uint32_t s = 0;
    for (int b = 0; b < 16; ++b) { hist[16 + b] = s; s += hist[b]; }
}

static __global__ void __launch_bounds__(BLOCK) k_order_scatter(SearchArgs a, uint32_t *hist, int32_t *perm)
{
    __shared__ uint32_t h[16], base[16];
    if (threadIdx.x < 16) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t b = 0, r = 0;
    if (q < (uint32_t)a.n_jobs) { b = order_bin(a, q); r = atomicAdd(&h[b], 1u); }
    __syncthreads();
    if (threadIdx.x < 16 && h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&hist[16 + threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (q < (uint32_t)a.n_jobs) perm[base[b] + r] = (int32_t)q;
}

// Strand-split mode, after k_search: per read, the rc strand's result if it has a hit,
// else the fwd strand's (bwtaln.c:343-359), else the splice fallback; the fwd search and
// its widths count as the reference's work only then.  A read whose deciding strand
// overflowed its lane goes to the next capacity pass whole (both strands, in order).
static __global__ void __launch_bounds__(BLOCK) k_split_finalize(SearchArgs a)
{
    const uint32_t q = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t n_jobs = a.n_dev ? (uint32_t)*a.n_dev : (uint32_t)a.n_jobs;
    unsigned long long q_add = 0, p_add = 0, w_add = 0;
    if (q < n_jobs) {
        const int job = a.job_list ? a.job_list[q] : (int)q;
        const int32_t nr = a.sp_n[2 * q], nf = a.sp_n[2 * q + 1];
        int32_t na = 0;
        uint32_t fl = 0;
        uint64_t off = 0;
        if (nr < 0 || (nr == 0 && nf < 0)) {
            fl = HSA_F_OVERFLOW;
            if (a.ovf_list) a.ovf_list[atomicAdd(&a.ctr[a.ovf_ctr], 1ull)] = job;
            else atomicAdd(&a.ctr[11], 1ull);
        } else if (nr > 0) {
            na = nr; off = a.sp_off[2 * q];
            q_add = a.sp_q[2 * q]; p_add = a.sp_p[2 * q];
        } else {
            w_add = a.wq[q];
            q_add = (unsigned long long)a.sp_q[2 * q] + a.sp_q[2 * q + 1] + w_add;
            p_add = (unsigned long long)a.sp_p[2 * q] + a.sp_p[2 * q + 1];
            if (nf > 0) { na = nf; off = a.sp_off[2 * q + 1]; }
            else fl = HSA_F_FALLBACK;
        }
        a.n_aln[job] = na;
        a.flags[job] = fl;
        a.hit_off[job] = off;
    }
    // one atomic per wave and counter
    for (int d = 32; d >= 1; d >>= 1) {
        q_add += __shfl_xor(q_add, d);
        p_add += __shfl_xor(p_add, d);
        w_add += __shfl_xor(w_add, d);
    }
    if ((threadIdx.x & 63) == 0) {
        if (q_add) atomicAdd(&a.ctr[2], q_add);
        if (p_add) atomicAdd(&a.ctr[4], p_add);
        if (w_add) { atomicAdd(&a.ctr[7], w_add); atomicAdd(&a.ctr[14], w_add); }
    }
}

// NT = lanes per workgroup: 256, or 64 when per-lane LDS (many buckets, long reads)
// would leave fewer than 16 waves per CU in 256-lane workgroups (plan_launch)
// HUGE: the last capacity pass (reads that overflowed the big pass): 32-bit pool
// links and popped slots reused through a free list, so a lane's pool holds any
// stack the reference can build (n_entries <= max_entries + 9, bwtgap.c:150-151).
template <int MW, bool GAPS, typename WT, int NT, bool HUGE = false, typename IT = uint32_t>
__global__ void __launch_bounds__(NT, HSA_WAVES_SIMD) k_search(SearchArgs a)
{
    using F = WFmt<WT>;
    using E = Ent<IT>;
    using CT = typename std::conditional<sizeof(IT) == 8, int64_t, int>::type;   // best_cnt (int in bwtgap.c:127)
    constexpr uint32_t HW = HitW<IT>::STAGE, OW = HitW<IT>::OUT;
    const IT TT = Ix<IT>::T(a);
    const IT *const CC = Ix<IT>::C(a);
    using LT = typename std::conditional<HUGE, uint32_t, uint16_t>::type;   // pool link
    // the helpers' code (SearchArgs::fr_*): gapped 32-bit searches only (configs 3 and 4, whose
    // small calls end in long strands); the other kernels stay as they were (their registers:
    // the 64-bit 4-bit-row kernels spilled with it)
    constexpr bool FRH = !HUGE && HSA_HELPERS && GAPS && sizeof(IT) == 4 && !WFmt<WT>::NIB;
    constexpr uint32_t NIL = HUGE ? 0xFFFFFFFFu : (uint32_t)NIL16;
#ifdef HSA_DIAG
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        g_diag[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memtime();
        g_diag[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    extern __shared__ __align__(16) uint8_t s_lds[];
    const uint32_t tid = threadIdx.x;
    const uint32_t gid = blockIdx.x * NT + tid;
    const int lane = (int)(tid & 63);
    // the two regimes' score tables (ntab entries each), then the two regimes
    for (uint32_t t = tid; t < 2 * a.ntab; t += NT) s_lds[t] = a.bmap[(t / a.ntab) * MAXS + t % a.ntab];
    static_assert(2 * sizeof(hsa_regime_t) <= 128, "regime LDS slot");
    hsa_regime_t *const s_reg = reinterpret_cast<hsa_regime_t *>(s_lds + 2 * a.ntab);
    if (tid < 2 * sizeof(hsa_regime_t) / 4)
        reinterpret_cast<uint32_t *>(s_reg)[tid] = reinterpret_cast<const uint32_t *>(a.regimes)[tid];
    __syncthreads();
    LT *const s_heads = reinterpret_cast<LT *>(s_lds + a.off_heads);
    using WTL = typename std::conditional<F::NIB, uint8_t, WT>::type;     // LDS element (8/16-bit formats)
    WTL *const s_wb = reinterpret_cast<WTL *>(s_lds + a.off_wb);
    WTL *const s_ws = reinterpret_cast<WTL *>(s_lds + a.off_ws);
    uint32_t *const s_nb = reinterpret_cast<uint32_t *>(s_lds + a.off_wb);   // 4-bit format: word q * NT + tid
    uint32_t *const s_ns = reinterpret_cast<uint32_t *>(s_lds + a.off_ws);
    // per-lane HBM scratch, wave-interleaved: element e of lane l of wave w at
    // (w * cap + e) * 64 + l, so one wave's accesses stay inside one small region
    // (few pages) and lanes at equal e coalesce
    const size_t wv = gid >> 6;
#if HSA_POOL_CHUNK
    const size_t link0 = wv * (size_t)((a.pcap + 31u) & ~31u) * 64 + (size_t)lane * 32;   // the lane's slot-0 link
#define NXT(s) reinterpret_cast<LT *>(a.nxt)[link0 + (size_t)((s) >> 5) * 2048 + ((s) & 31u)]
#else
    const size_t link0 = wv * a.pcap * 64 + (size_t)lane;        // the lane's slot-0 link
#define NXT(s) reinterpret_cast<LT *>(a.nxt)[link0 + (size_t)(s) * 64]
#endif
    const size_t pbase = pool_base<IT>(wv, a.pcap, lane);        // ... and slot-0 pool entry
#define HB(i) r->hbuf[(wv * r->hcap * HW + (uint32_t)(i)) * 64 + lane]   // r = cold_args() in scope
#define HEAD(b) s_heads[(uint32_t)(b) * NT + tid]
    // pruning elements in LDS, word-interleaved: the word holding elements
    // [EPW*q, EPW*q + EPW) of a lane is word q * NT + tid, so every lane reads its
    // own bank whatever position it is at, and a row copies in one store per word
#define WB(p) s_wb[(((uint32_t)(p) / F::EPW) * NT + tid) * F::EPW + (uint32_t)(p) % F::EPW]
#define WS(p) s_ws[(((uint32_t)(p) / F::EPW) * NT + tid) * F::EPW + (uint32_t)(p) % F::EPW]
#define RG(f) (s_reg[C_REG(ctl)].f)

    // ---- persistent per-lane state
    uint32_t ctl = PH_IDLE;        // control word (C_* accessors)
    uint32_t qpos = 0;             // position of the read in the job list (width row = qpos * 2 + strand)
    uint32_t pen = 0;              // s_mm | s_gapo << 10 | s_gape << 20
    uint32_t rmode = 0;            // mode | max_gapo << 8 | max_gape << 16
    uint32_t pos = 0;              // exact tail: next position
    IT ik = 0, il = 0;             // exact-tail interval
    IT aux = 0;                    // exact tail: rev_l
    int opt_max_diff = 0, max_diff = 0, best_score = 0, n_aln = 0, n_entries = 0;
    CT best_cnt = 0;
    uint32_t pool_top = 0;
    uint32_t free_head = NIL;      // HUGE: popped slots, linked through NXT
    uint32_t idle_acc = 0;         // (A): lane-iterations the waiting lanes idled since the last batch
    BMask<MW> mask;
    // the current entry (k, l, rev_k, meta); between an expansion and the next pop
    // it holds the virtual top when C_VT is set (the last child pushed, when it is
    // the next pop: it never goes to the pool)
    E e{0, 0, 0, 0};
    // per-lane statistics (a lane's counts of one launch stay far below 2^32); kept in
    // VGPRs: wave-uniform accumulators pushed the kernel's SGPRs into spills
    uint32_t st_p = 0, st_wq = 0, st_q = 0, st_b = 0;
    uint32_t sq0 = 0, sp0 = 0;            // split mode: the counters when the item started
    // helpers (SearchArgs::fr_*): frs bit 0 the strand offered its frontier (owner), bit 1
    // this lane runs a sub-search, bit 2 no more offers from this strand; fr_p0 the pops at
    // the strand's start, then at the offer (owner) or the sub-search's start (helper), with
    // fr_q0 the rank queries at that point
    uint32_t frs = 0, fr_p0 = 0, fr_q0 = 0;
    uint32_t fr_tick = 0;          // the wave's iterations (waiting lanes poll every 128)
    uint32_t st_hs = 0, st_hq = 0; // sub-searches this lane ran, and their rank queries
    const uint32_t n_jobs = a.n_dev ? (uint32_t)*a.n_dev : (uint32_t)a.n_jobs;
#ifdef HSA_DIAG
    uint32_t dc[21] = {0};
    uint64_t tsec[4] = {0, 0, 0, 0};
    uint64_t tt = 0;
    uint64_t rd_t0 = 0;
    uint32_t rd_steps = 0, rd_p0 = 0;
#define TMARK(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); tsec[k] += t_ - tt; tt = t_; } while (0)
#endif

#define S_MM ((int)(pen & 1023u))
#define S_GO ((int)((pen >> 10) & 1023u))
#define S_GE ((int)(pen >> 20))
#define R_MODE ((int)(rmode & 255u))
#define R_MAXGO ((int)((rmode >> 8) & 255u))
#define R_MAXGE ((int)(rmode >> 16))
#define SCORE(mm, go, ge) ((mm) * S_MM + (go) * S_GO + (ge) * S_GE)

    // pruning elements of the read row / seed row at p (WFmt), and the element write of gap_shadow
    auto wbg = [&](int p) -> uint32_t {
        if constexpr (F::NIB) return (s_nb[((uint32_t)p >> 3) * NT + tid] >> (((uint32_t)p & 7u) * 4u)) & 15u;
        else return WB(p);
    };
    auto wsg = [&](int p) -> uint32_t {
        if constexpr (F::NIB) return (s_ns[((uint32_t)p >> 3) * NT + tid] >> (((uint32_t)p & 7u) * 4u)) & 15u;
        else return WS(p);
    };
    auto wbs = [&](int p, uint32_t v) {
        if constexpr (F::NIB) {
            uint32_t &w = s_nb[((uint32_t)p >> 3) * NT + tid];
            const uint32_t sh = ((uint32_t)p & 7u) * 4u;
            w = (w & ~(15u << sh)) | v << sh;
        } else {
            WB(p) = (WTL)v;
        }
    };
    // 4-bit format: the strand's 8-bit HBM row (base codes), and the base the next
    // step needs, loaded in the control phase so that its latency overlaps the rank load
    const uint8_t *rowp = nullptr;
    uint32_t cur_c = 0;
    // 4-bit format: the row word (4 positions) the last base came from, kept in registers.
    // A strand's steps walk its positions downwards (the virtual top is the child at
    // i - 1, an exact tail steps pos--), so most bases come from the word already held:
    // a row load is one L2 request (the rows of the resident waves are far larger than
    // L2 and mostly missed it), and the search is request-rate bound (config 5: 1.40 L2
    // requests per rank query with a load per step, 0.97 in config 2's 8-bit rows).
#ifndef HSA_ROWCACHE
#define HSA_ROWCACHE 1                     // A/B builds: -DHSA_ROWCACHE=0 loads the byte every step
#endif
    uint32_t rw_q = 0xFFFFFFFFu, rw_w = 0;
    // base of the current strand's sequence at p (from the LDS element, or the HBM row)
    auto getc = [&](int p) -> uint32_t {
        if constexpr (F::NIB && !HSA_ROWCACHE) {
            return WFmt<uint8_t>::code(rowp[((uint32_t)p >> 2) * 256u + ((uint32_t)p & 3u)]);
        } else if constexpr (F::NIB) {
            const uint32_t q = (uint32_t)p >> 2;
            if (q != rw_q) {
                rw_w = *reinterpret_cast<const uint32_t *>(rowp + q * 256u);
                rw_q = q;
            }
            return WFmt<uint8_t>::code((rw_w >> (((uint32_t)p & 3u) * 8u)) & 0xFFu);
        } else {
            return F::code(WB(p));
        }
    };
    // stack bucket of an entry: dense index of its score (bwtgap.c:46-75)
    auto bucket_of = [&](uint32_t m) -> int {
        if (!GAPS && a.mm_buckets) return M_MM(m);
        const int sc = SCORE(M_MM(m), M_GO(m), M_GE(m));
        return (uint32_t)sc < a.ntab ? (int)s_lds[C_REG(ctl) * a.ntab + sc] : 0xFF;
    };
    // push to the pool (gap_push, bwtgap.c:46-75)
    auto flush = [&](const E &v, int b) {
        if ((uint32_t)b >= a.nb) { ctl |= 1u << 8; return; }
        uint32_t slot;
        if (HUGE && free_head != NIL) {
            slot = free_head;
            free_head = NXT(slot);
        } else {
            if (pool_top >= a.pcap) { ctl |= 1u << 8; return; }
            slot = pool_top++;
        }
        DC(8);
        ent_store<IT>(a.pool, pbase, slot, v);
        const uint32_t old = mask.test(b) ? (uint32_t)HEAD(b) : NIL;
        NXT(slot) = (LT)old;
        HEAD(b) = (LT)slot;
        mask.set(b);
    };
    auto start_search = [&]() {
        best_score = SCORE(opt_max_diff + 1, R_MAXGO + 1, R_MAXGE + 1);
        max_diff = opt_max_diff;
        best_cnt = 0; n_aln = 0;
        mask.clear(); pool_top = 0; free_head = NIL;
        e = E{0, TT, 0, meta_pack((uint32_t)C_LEN(ctl), ST_M, 0, 0, 0, 0)};   // root (bwtgap.c:142)
        ctl |= 1u << 6;
        n_entries = 1;
        frs = 0; fr_p0 = st_p;
        SET_PH(ctl, PH_POP);
    };
    // the item number of the strand this lane searches (split mode: list position * 2 + 1 for fwd)
    auto fr_key = [&]() -> uint32_t { return qpos * 2u + (1u - C_STRAND(ctl)); };
    // width row of the current strand: row qpos * 2 + strand, 64 rows interleaved
    auto row_base = [&](uint32_t cap_words) -> size_t {
        const int32_t *const rm = cold_args()->rmap;
        const uint32_t r = rm ? (C_STRAND(ctl) ? qpos : (uint32_t)rm[qpos]) : qpos * 2u + C_STRAND(ctl);
        return (size_t)(r >> 6) * cap_words * 64 + (r & 63u);
    };
    // copy the strand's pruning elements (k_widths) into the lane's LDS columns, then
    // start bwt_match_gap (bwtgap.c:141-142)
    auto start_strand = [&]() {
        // LDS-DMA (global_load_lds_dword): word q of every active lane lands at
        // word q * NT + tid, which is exactly the wave's slice of the LDS layout, so
        // the whole row is in flight at once and one wait covers it
        const ColdArgs r = cold_args();
        const uint32_t *src = reinterpret_cast<const uint32_t *>(r->wb) + row_base(r->rb / 4);
        const uint32_t nwb = r->rb / 4;                // row capacity in words (uniform)
        if constexpr (F::NIB) {
            // two 8-bit words per LDS word, eight loads in flight
            rowp = reinterpret_cast<const uint8_t *>(src);
            rw_q = 0xFFFFFFFFu;
            auto pack = [&](const uint32_t *row, uint32_t nw, uint32_t *dst, uint32_t cap) {
                const uint32_t nn = (nw + 1u) / 2u < cap ? (nw + 1u) / 2u : cap;   // LDS words of the row
                for (uint32_t j = 0; j < nn; j += 4) {
                    uint32_t w[8];
#pragma unroll
                    for (uint32_t u = 0; u < 8; ++u) w[u] = 2u * j + u < nw ? row[(2u * j + u) * 64u] : 0u;
#pragma unroll
                    for (uint32_t u = 0; u < 4; ++u)
                        if (j + u < nn) dst[(j + u) * NT + tid] = nib4(w[2u * u]) | nib4(w[2u * u + 1u]) << 16;
                }
            };
            pack(src, nwb, s_nb, r->nib_wb);
            if (C_SEED(ctl) && !C_ALIAS(ctl))
                pack(reinterpret_cast<const uint32_t *>(r->ws) + row_base(r->rs / 4), r->rs / 4, s_ns, r->nib_ws);
        } else {
        uint32_t *const db = reinterpret_cast<uint32_t *>(s_wb) + (tid & ~63u);
        for (uint32_t q = 0; q < nwb; ++q)
            __builtin_amdgcn_global_load_lds(src + q * 64, db + q * NT, 4, 0, 0);
        if (C_SEED(ctl) && !C_ALIAS(ctl)) {
            const uint32_t *ss = reinterpret_cast<const uint32_t *>(r->ws) + row_base(r->rs / 4);
            uint32_t *const ds = reinterpret_cast<uint32_t *>(s_ws) + (tid & ~63u);
            const uint32_t nws = r->rs / 4;
            for (uint32_t q = 0; q < nws; ++q)
                __builtin_amdgcn_global_load_lds(ss + q * 64, ds + q * NT, 4, 0, 0);
        }
        }
        __builtin_amdgcn_s_waitcnt(0);                 // the DMA writes are visible to LDS reads
        DC(15);
        start_search();
    };
    auto finish_job = [&](uint32_t fl, int na, uint64_t ho) {
        const ColdArgs r = cold_args();
#ifdef HSA_DIAG
        atomicMax(&g_dctr[21], (unsigned long long)rd_steps);
        atomicMax(&g_dctr[22], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - rd_t0));
        atomicMax(&g_dctr[23], (unsigned long long)(st_p - rd_p0));
        atomicMax(&g_dctr[na > 0 ? 24 : 25], (unsigned long long)rd_steps);
#endif
        if (r->split) {                       // one strand of a read: k_split_finalize decides
            const uint32_t pi = qpos * 2u + (1u - C_STRAND(ctl));
            r->sp_n[pi] = (fl & HSA_F_OVERFLOW) ? -1 : na;
            r->sp_off[pi] = ho;
            r->sp_q[pi] = st_q - sq0;
            r->sp_p[pi] = st_p - sp0;
            st_q = sq0; st_p = sp0;
            if constexpr (FRH) {
                if (a.fr_budget) {
                    if (frs & 1u) atomicOr(&r->fr_st[pi], FR_DONE);   // its helpers stop
                    atomicAdd(&r->fr_c[2], 1ull);                      // items finished (the exit test)
                    frs = 0;
                }
            }
            SET_PH(ctl, PH_IDLE);
            return;
        }
        const int job = r->job_list ? r->job_list[qpos] : (int)qpos;
        if (fl & HSA_F_NEEDFWD) {                 // the forward pass writes its outputs
            r->fwd_list[atomicAdd(r->fwd_n, 1ull)] = job;
            SET_PH(ctl, PH_IDLE);
            return;
        }
        if (fl & HSA_F_OVERFLOW) {
            if (r->ovf_list) r->ovf_list[atomicAdd(&r->ctr[r->ovf_ctr], 1ull)] = job;   // re-run by the next pass
            else atomicAdd(&r->ctr[11], 1ull);                                  // the last pass: stays unfinished
        }
        r->n_aln[job] = na;
        r->flags[job] = fl;
        r->hit_off[job] = ho;
        SET_PH(ctl, PH_IDLE);
    };
    // a sub-search ends (no hit, a hit, its item decided, or its entries offered on): its
    // work goes to the item's sums, then its count leaves the item's open sub-searches
    auto help_done = [&]() {
        const ColdArgs r = cold_args();
        const uint32_t key = fr_key();
        const unsigned long long dq = st_q - fr_q0, dp = st_p - fr_p0;
        st_q = fr_q0; st_p = fr_p0;
        const unsigned long long o1 = atomicAdd(&r->fr_q[key], dq), o2 = atomicAdd(&r->fr_p[key], dp);
        asm volatile("s_waitcnt vmcnt(0)" :: "v"(o1), "v"(o2) : "memory");   // the sums land first
        atomicSub(&r->fr_st[key], 1u);
        ++st_hs; st_hq += (uint32_t)dq;
        frs = 0;
        SET_PH(ctl, PH_IDLE);
    };
    auto end_strand = [&]() {
        if constexpr (FRH) {
            if (frs & 2u) { help_done(); return; }
        }
        if (n_aln > 0) {
            const ColdArgs r = cold_args();
            const unsigned long long o = atomicAdd(&r->ctr[1], (unsigned long long)n_aln);
            if (o + (uint64_t)n_aln > r->hit_cap) { finish_job(HSA_F_OVERFLOW, 0, 0); return; }
            uint32_t *dst = r->hits + o * OW;
            const uint32_t s30 = C_STRAND(ctl) << 30;
            for (int h = 0; h < n_aln; ++h) {
                // bwtaln.c:371-372 (a direct bwt_match_gap call leaves start/end 0)
                const uint32_t end = h == 0 && !r->mg ? (uint32_t)(C_LEN(ctl) - 1) : 0u;
                if constexpr (sizeof(IT) == 4) {
                    // the six staged words first, then the record: one memory round trip per hit
                    const uint32_t v0 = HB(h * 9 + 0), v1 = HB(h * 9 + 1), v2 = HB(h * 9 + 2), v3 = HB(h * 9 + 3),
                                   v4 = HB(h * 9 + 4), v8 = HB(h * 9 + 8);
                    dst[h * 9 + 0] = v0;
                    dst[h * 9 + 1] = v1;
                    dst[h * 9 + 2] = v2;
                    dst[h * 9 + 3] = v3;
                    dst[h * 9 + 4] = v4;
                    dst[h * 9 + 5] = s30;
                    dst[h * 9 + 6] = 0;
                    dst[h * 9 + 7] = end;
                    dst[h * 9 + 8] = v8;
                } else {
                    // hsa_aln64_t (include/hsa_gpu.h): 14 words
                    uint32_t v[10];
#pragma unroll
                    for (int j = 0; j < 10; ++j) v[j] = HB(h * 10 + j);
                    dst[h * 14 + 0] = v[0];
                    dst[h * 14 + 1] = s30;
#pragma unroll
                    for (int j = 1; j < 9; ++j) dst[h * 14 + 1 + j] = v[j];
                    dst[h * 14 + 10] = 0;
                    dst[h * 14 + 11] = end;
                    dst[h * 14 + 12] = v[9];
                    dst[h * 14 + 13] = 0;
                }
            }
            finish_job(0, n_aln, o);
        } else if (cold_args()->mg || cold_args()->split) {
            finish_job(0, 0, 0);        // one call (or one split item), one strand
        } else if (C_STRAND(ctl)) {
            const uint32_t wq = cold_args()->wq[qpos];
            if (wq == HSA_NOFWD) {
                finish_job(HSA_F_NEEDFWD, 0, 0);   // its forward row is computed by the forward pass
            } else {
                ctl &= ~(1u << 3);          // strand 0
                st_wq += wq;                // its widths are the reference's work now (bwtaln.c:344-348)
                start_strand();
            }
        } else {
            finish_job(HSA_F_FALLBACK, 0, 0);
        }
    };
    // hit handling (bwtgap.c:188-243) for entry e with final interval (k,l,rk,rl);
    // returns false when the search must stop
    auto on_hit = [&](IT k, IT l, IT rk, IT rl) -> bool {
        const ColdArgs r = cold_args();
        if constexpr (FRH) {
            if (frs & 3u) {
                atomicOr(&r->fr_st[fr_key()], FR_HIT);   // the item has a hit: its sub-searches stop
                if (frs & 2u) return false;              // a helper records nothing
            }
        }
        const uint32_t m = e.w;
        const int score = SCORE(M_MM(m), M_GO(m), M_GE(m));
        if (n_aln == 0) {
            best_score = score;
            const int best_diff = M_MM(m) + M_GO(m) + ((R_MODE & MODE_GAPE) ? M_GE(m) : 0);
            if (!(R_MODE & MODE_NONSTOP)) max_diff = (best_diff + 1 > opt_max_diff) ? opt_max_diff : best_diff + 1;
        }
        if (score == best_score) {
            if constexpr (sizeof(IT) == 4) best_cnt = (int)((uint32_t)best_cnt + (l - k + 1u));
            else best_cnt += (CT)(l - k + 1u);
        } else if (best_cnt > RG(max_top2)) {
            return false;
        }
        bool add = true;
        if (M_GO(m)) {
            for (int j = 0; j < n_aln; ++j) {
                if constexpr (sizeof(IT) == 4) {
                    if (HB(j * 9 + 1) == k && HB(j * 9 + 2) == l) { add = false; break; }
                } else {
                    const uint64_t hk = (uint64_t)HB(j * 10 + 1) | (uint64_t)HB(j * 10 + 2) << 32;
                    const uint64_t hl = (uint64_t)HB(j * 10 + 3) | (uint64_t)HB(j * 10 + 4) << 32;
                    if (hk == k && hl == l) { add = false; break; }
                }
            }
        }
        if (add) {
            if ((uint32_t)n_aln >= r->hcap) { ctl |= 1u << 8; return false; }
            // gap_shadow (bwtgap.c:94-105) on width_back[0, last_diff_pos), then the
            // pruning elements of those positions (eq bit of p needs w[p+1])
            const IT x = l - k + 1u;
            const int ldp = M_ISD(m) ? M_I(m) : 0;
            if (ldp > 0) {
#ifdef HSA_DIAG
                DC(13); dc[14] += (uint32_t)ldp;
#endif
                IT *const wg = reinterpret_cast<IT *>(r->wg) + row_base(r->rg);
                int32_t *const wd = r->wbid ? r->wbid + row_base(r->rg) : nullptr;
#define WG(p) wg[(uint32_t)(p) * 64]
                IT jj = 0;
                for (int p = 0; p < ldp; ++p) {
                    IT w = WG(p);
                    if (w > x) { w -= x; WG(p) = w; }
                    else if (w == x) {
                        wbs(p, (wbg(p) & ~F::BIDM) | 1u);
                        WG(p) = TT - (++jj);
                        if (wd) wd[(uint32_t)p * 64] = 1;
                    }
                }
                IT wnext = WG(ldp);
                for (int p = ldp - 1; p >= 0; --p) {
                    const IT w = WG(p);
                    wbs(p, (wbg(p) & ~F::EQ) | (w == wnext ? F::EQ : 0u));
                    wnext = w;
                }
#undef WG
            }
            const uint32_t mw = (uint32_t)M_MM(m) | (uint32_t)M_GO(m) << 16 | (uint32_t)M_GE(m) << 24;
            if constexpr (sizeof(IT) == 4) {
                HB(n_aln * 9 + 0) = mw;
                HB(n_aln * 9 + 1) = k; HB(n_aln * 9 + 2) = l; HB(n_aln * 9 + 3) = rk; HB(n_aln * 9 + 4) = rl;
                HB(n_aln * 9 + 8) = (uint32_t)score;
            } else {
                HB(n_aln * 10 + 0) = mw;
                HB(n_aln * 10 + 1) = (uint32_t)k; HB(n_aln * 10 + 2) = (uint32_t)(k >> 32);
                HB(n_aln * 10 + 3) = (uint32_t)l; HB(n_aln * 10 + 4) = (uint32_t)(l >> 32);
                HB(n_aln * 10 + 5) = (uint32_t)rk; HB(n_aln * 10 + 6) = (uint32_t)(rk >> 32);
                HB(n_aln * 10 + 7) = (uint32_t)rl; HB(n_aln * 10 + 8) = (uint32_t)(rl >> 32);
                HB(n_aln * 10 + 9) = (uint32_t)score;
            }
            ++n_aln;
        }
        return true;
    };
    // m (available differences) of entry e (bwtgap.c:160-163)
    auto m_of = [&](uint32_t m) -> int {
        int mm = max_diff - (M_MM(m) + M_GO(m));
        if (R_MODE & MODE_GAPE) mm -= M_GE(m);
        return mm;
    };

    // start work item `item` (a read, a strand in split mode, or a direct call)
    auto begin_item = [&](uint32_t item) {
        const ColdArgs r = cold_args();
#ifdef HSA_DIAG
        rd_t0 = __builtin_amdgcn_s_memrealtime(); rd_steps = 0; rd_p0 = st_p;
#endif
        qpos = r->split ? item >> 1 : item;
        if (r->perm) qpos = (uint32_t)r->perm[qpos];
        const int job = r->job_list ? r->job_list[qpos] : (int)qpos;
        const hsa_job_t J = r->jobs[job];
        opt_max_diff = J.max_diff;
        const uint32_t len = J.len;
        if (r->mg) {
            // one direct bwt_match_gap call: its strand, its width_seed kind
            // (host-checked: 0 <= seed_len <= len when width_seed is given)
            const hsa_mg_job_t M = r->mg[job];
            const uint32_t has_seed = M.seed != HSA_SEED_NONE;
            ctl = (uint32_t)(M.strand & 1) << 3 | has_seed << 4 | (uint32_t)(J.regime & 1) << 5 |
                  (M.seed == HSA_SEED_ALIAS ? 1u : 0u) << 7 | len << 10 |
                  (has_seed ? (uint32_t)J.seed_len : 0u) << 20;
        } else {
            const uint32_t has_seed = (int)len > J.seed_len;
            ctl = 8u | has_seed << 4 | (uint32_t)(J.regime & 1) << 5 | len << 10 |
                  (has_seed ? (uint32_t)J.seed_len : 0u) << 20;     // strand 1 (rc first, bwtaln.c:343)
            if ((r->split && (item & 1u)) || r->fwd_only) ctl &= ~8u;   // split: odd items search fwd
            sq0 = st_q; sp0 = st_p;
        }
        const hsa_regime_t *R = s_reg + (J.regime & 1);
        pen = (uint32_t)R->s_mm | (uint32_t)R->s_gapo << 10 | (uint32_t)R->s_gape << 20;
        rmode = (uint32_t)R->mode | (uint32_t)R->max_gapo << 8 | (uint32_t)R->max_gape << 16;
        if (opt_max_diff > R->max_diff) ctl |= 2u << 8;
        start_strand();
    };
    // helpers: publish this strand's live entries -- the virtual top, then every bucket's
    // list -- as sub-search roots of its item.  An entry's words are stored at agent scope
    // and its tag after a release, and the item's open-sub-search count is raised first, so
    // the count never reaches zero while one of them is unsearched.  False (nothing
    // published): the frontier is full, or the lists do not add up to n_entries.
    auto fr_offer = [&]() -> bool {
        const ColdArgs r = cold_args();
        const uint32_t cnt = (uint32_t)n_entries, nch = (cnt + FR_CH - 1u) / FR_CH;
        unsigned long long o = __hip_atomic_load(&r->fr_c[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {                                       // reserve nch chunks (no walk when they do not fit)
            if (o + nch > (unsigned long long)r->fr_cap) { atomicAdd(&r->fr_c[5], 1ull); return false; }
            const unsigned long long w = atomicCAS(&r->fr_c[0], o, o + nch);
            if (w == o) break;
            o = w;
        }
        const uint32_t key = fr_key();
        const unsigned int pend = atomicAdd(&r->fr_st[key], nch);     // before any chunk is published
        asm volatile("s_waitcnt vmcnt(0)" :: "v"(pend) : "memory");
        auto put = [&](uint32_t j, const E &v) {      // two 16-byte stores (the release below covers them)
            uint4 *d = reinterpret_cast<uint4 *>(r->fr_ent + ((o + j / FR_CH) * FR_CH + j % FR_CH) * FR_EW);
            if constexpr (sizeof(IT) == 4) {
                d[0] = make_uint4(v.x, v.y, v.z, v.w);
            } else {
                d[0] = make_uint4((uint32_t)v.x, (uint32_t)(v.x >> 32), (uint32_t)v.y, v.w);
                d[1] = make_uint4((uint32_t)(v.y >> 32), (uint32_t)v.z, (uint32_t)(v.z >> 32), 0u);
            }
        };
        uint32_t j = 0;
        if (C_VT(ctl)) put(j++, e);
        {
            BMask<MW> mm = mask;
            while (mm.any() && j < cnt) {
                const int b = mm.lowest();
                mm.reset(b);
                for (uint32_t sl = HEAD(b); sl != NIL && j < cnt; sl = NXT(sl)) put(j++, ent_load<IT>(a.pool, pbase, sl));
            }
        }
        // the lists must hold exactly n_entries: otherwise publish what was written, and mark
        // the item as having a hit, so that nothing is concluded from its sub-searches
        if (j != cnt) atomicOr(&r->fr_st[key], FR_HIT);
        for (uint32_t c = 0; c < nch; ++c) {
            const uint32_t in = j > c * FR_CH ? (j - c * FR_CH < FR_CH ? j - c * FR_CH : FR_CH) : 0u;
            r->fr_tag[o + c] = in << 26 | (key + 1u);
        }
        // complete chunks only enter the ready queue: a taker never waits on a walk
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long q0 = atomicAdd(&r->fr_c[9], (unsigned long long)nch);
        for (uint32_t c = 0; c < nch; ++c)
            __hip_atomic_store(&r->fr_rq[q0 + c], (uint32_t)(o + c) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&r->fr_c[4], 1ull);
        return true;
    };
    // helpers: a waiting lane starts a sub-search at ready-queue position qp: the chunk's
    // entries go to the lane's own stack (their order does not matter before a hit), under
    // its item's row and regime.  The queue slot is written right after the tail moved; the
    // chunk itself was released before that (agent-scope acquire, then plain loads).
    auto help_start = [&](unsigned long long qp) {
        const ColdArgs r = cold_args();
        uint32_t c1;
        while ((c1 = __hip_atomic_load(&r->fr_rq[qp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const size_t c = c1 - 1u;
        const uint32_t t = r->fr_tag[c];
        begin_item((t & 0x3FFFFFFu) - 1u);               // its strand's row and regime, a fresh stack
        ctl &= ~(1u << 6);                               // no virtual top: every entry from the pool
        const uint32_t in = t >> 26;
        const uint4 *s4 = reinterpret_cast<const uint4 *>(r->fr_ent + c * FR_CH * FR_EW);
        for (uint32_t q = 0; q < in; ++q) {
            const uint4 u = s4[2 * q], w = s4[2 * q + 1];
            E v;
            if constexpr (sizeof(IT) == 4) {
                v.x = u.x; v.y = u.y; v.z = u.z;
            } else {
                v.x = (uint64_t)u.x | (uint64_t)u.y << 32;
                v.y = (uint64_t)u.z | (uint64_t)w.x << 32;
                v.z = (uint64_t)w.y | (uint64_t)w.z << 32;
            }
            v.w = u.w;
            flush(v, bucket_of(v.w));
        }
        n_entries = (int)in;
        frs = 2u; fr_p0 = st_p; fr_q0 = st_q;
    };
    // helpers: the waiting lanes of the wave take published chunks (one CAS for the wave), or
    // leave once every item has finished and every chunk was taken (a sub-search still
    // running then belongs to a finished item, and stops at its next poll)
    auto fr_take = [&]() {
        const uint64_t wb = __ballot(C_PH(ctl) == PH_WAIT);
        if (!wb) return;
        const ColdArgs r = cold_args();
        const int leader = __ffsll((unsigned long long)wb) - 1;
        unsigned long long t0 = 0;
        uint32_t k = 0, fin = 0;
        if (lane == leader) {
            const unsigned long long want = (unsigned long long)__popcll(wb);
            unsigned long long tk = __hip_atomic_load(&r->fr_c[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long rs = __hip_atomic_load(&r->fr_c[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tk < rs) {
                for (int tries = 0; tries < 4 && tk < rs; ++tries) {     // (lost races: the next poll)
                    const unsigned long long kk = rs - tk < want ? rs - tk : want;
                    const unsigned long long w = atomicCAS(&r->fr_c[1], tk, tk + kk);
                    if (w == tk) { t0 = tk; k = (uint32_t)kk; break; }
                    tk = w;
                }
                if (k) atomicSub(&r->fr_c[3], (unsigned long long)k);
            } else if (__hip_atomic_load(&r->fr_c[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                           (unsigned long long)n_jobs * 2ull &&
                       __hip_atomic_load(&r->fr_c[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                           __hip_atomic_load(&r->fr_c[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                // every item has finished (none can offer more) and every reserved chunk was taken
                fin = 1;
                atomicSub(&r->fr_c[3], want);
            }
        }
        t0 = __shfl(t0, leader); k = __shfl(k, leader); fin = __shfl(fin, leader);
        if (C_PH(ctl) == PH_WAIT) {
            const uint32_t rank = (uint32_t)__popcll(wb & ((1ull << lane) - 1ull));
            if (rank < k) help_start(t0 + rank);
            else if (fin) SET_PH(ctl, PH_EXIT);
        }
    };

#ifdef HSA_DIAG
    tt = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
        ++fr_tick;
        // ---------------- (A) strand ends and read acquisition, batched per wave.
        // The rare steps of a read -- copying its hits out (end_strand), the switch to
        // the forward strand with its row DMA, taking the next read -- are long code
        // paths that the whole wave executes whenever one lane needs one.  A lane that
        // reaches one waits (PH_END / PH_IDLE) and the wave then runs each path once for
        // all waiting lanes, when running it costs less than the waiting has (ski
        // rental): once the waiting lanes have idled batch_idle lane-iterations since
        // the last run (or batch_k lanes wait, or no lane is searching).  Reads that end
        // often (config 2: ~430 pops per read) gather ~16 waiters first; long gapped
        // searches (config 3: ~6 600 pops) run it with a few, instead of idling lanes
        // for hundreds of iterations.
        const uint64_t wm = __ballot(C_PH(ctl) == PH_IDLE || C_PH(ctl) == PH_END);
        idle_acc += (uint32_t)__popcll(wm);
        const bool none_searching = __ballot(C_PH(ctl) != PH_EXIT && C_PH(ctl) != PH_IDLE && C_PH(ctl) != PH_END &&
                                             C_PH(ctl) != PH_WAIT) == 0;
        if (wm && (idle_acc >= a.batch_idle || (uint32_t)__popcll(wm) >= a.batch_k || none_searching)) {
            idle_acc = 0;
            if (C_PH(ctl) == PH_END) end_strand();
            const bool need = C_PH(ctl) == PH_IDLE;
            const uint64_t mb = __ballot(need);
            if (mb) {
                const int leader = __ffsll((unsigned long long)mb) - 1;
                unsigned long long base = 0;
                const ColdArgs r = cold_args();
                if (lane == leader) base = atomicAdd(&r->ctr[r->qctr], (unsigned long long)__popcll(mb));
                base = __shfl(base, leader);
                {
                    const unsigned long long j = base + (unsigned long long)__popcll(mb & ((1ull << lane) - 1ull));
                    const bool got = need && j < (unsigned long long)n_jobs << (r->split ? 1 : 0);
                    if constexpr (FRH) {
                        if (a.fr_budget) {             // the lanes that found the queue empty wait for entries
                            const uint32_t nf = (uint32_t)(__popcll(mb) - __popcll(__ballot(got)));
                            if (lane == leader && nf) atomicAdd(&r->fr_c[3], (unsigned long long)nf);
                        }
                    }
                    if (need) {
                        if (got) begin_item((uint32_t)j);
                        else SET_PH(ctl, (FRH && a.fr_budget) ? PH_WAIT : PH_EXIT);
                    }
                }
            }
            if constexpr (FRH) {
                if (a.fr_budget) fr_take();
            }
        } else if constexpr (FRH) {
            // waiting lanes beside searching ones look for entries every 128 iterations (a poll
            // is a dependent load the whole wave waits for); a wave with none searching, every
            // iteration, after a sleep
            if (a.fr_budget && (none_searching || (fr_tick & 127u) == 64u)) fr_take();
        }
        if (__all(C_PH(ctl) == PH_EXIT)) break;
        if constexpr (FRH) {
            if (a.fr_budget && __ballot(C_PH(ctl) != PH_WAIT && C_PH(ctl) != PH_EXIT) == 0) {
#pragma unroll
                for (int z = 0; z < 4; ++z) __builtin_amdgcn_s_sleep(127);
            }
        }

#ifdef HSA_DIAG
        TMARK(0);
#endif
        // ---------------- (B) control until a rank step is needed
        // req: 1 a rank pair at rp1, rp2
        int req = 0;
        IT rp1 = 0, rp2 = 0;
#ifdef HSA_DIAG
        if (lane == 0) DC(5);
#endif
        // One control pass per iteration: a lane whose pop needs no rank step (pruned,
        // hit, strand change) just skips this iteration's step instead of making the whole
        // wave run the control code again.
        if (C_PH(ctl) != PH_EXIT && C_PH(ctl) != PH_IDLE && C_PH(ctl) != PH_END && C_PH(ctl) != PH_WAIT) do {
#ifdef HSA_DIAG
            { const uint64_t em = __ballot(1); if (lane == __ffsll((unsigned long long)em) - 1) DC(7); }
#endif
            if (C_OVF(ctl)) {
                if constexpr (FRH) {
                    if (frs & 2u) {       // a sub-search outgrew the lane: no proof, the owner searches on
                        atomicOr(&cold_args()->fr_st[fr_key()], FR_HIT);
                        help_done();
                        break;
                    }
                }
                if (C_OVF(ctl) > 1) atomicAdd(&cold_args()->ctr[5], 1ull);
                finish_job(HSA_F_OVERFLOW, 0, 0);
                break;
            }
            const uint32_t ph = C_PH(ctl);
            if (ph == PH_EXACT) {
                if constexpr (F::NIB) {
                    // the rank step goes out with the base load; an N (c > 3) drops it in (D)
                    cur_c = getc((int)pos);
                    req = 1; rp1 = ik; rp2 = il + 1u;
                    break;
                }
                const uint32_t c = getc((int)pos);
                if (c > 3) { SET_PH(ctl, PH_POP); continue; }              // 2BWT-Interface.c:377
                req = 1; rp1 = ik; rp2 = il + 1u;
                break;
            }
            // PH_POP: bwtgap.c:144-186
            if (n_entries == 0 || n_entries > RG(max_entries)) { SET_PH(ctl, PH_END); continue; }
            if constexpr (FRH) {
                // helpers, every 16 pops of a strand: a sub-search stops once its item is decided
                // (a hit, or its owner ended); an owner whose offered entries have all been
                // searched without a hit has its answer -- no hit -- and its work: what it did
                // before the offer plus its sub-searches'.  Every 64 pops past fr_budget, a strand
                // with no hit yet offers its entries while more lanes wait than entries do.
                // (the polls run on the wave's iteration count, so that all its lanes load
                // together: a lane's own cadence made some lane of the wave wait on a load
                // nearly every iteration)
                const uint32_t ps = st_p - fr_p0;
                if (a.fr_budget && (fr_tick & 31u) == 0u) {
                    const ColdArgs r = cold_args();
                    bool stop = false;
                    if (frs & 3u) {
                        const uint32_t key = fr_key();
                        const uint32_t sv = __hip_atomic_load(&r->fr_st[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (frs & 2u) {
                            stop = (sv & (FR_HIT | FR_DONE)) != 0u;
                        } else if (sv == 0u && n_aln == 0) {
                            st_q = fr_q0 + (uint32_t)atomicAdd(&r->fr_q[key], 0ull);
                            st_p = fr_p0 + (uint32_t)atomicAdd(&r->fr_p[key], 0ull);
                            atomicAdd(&r->fr_c[7], 1ull);
                            stop = true;
                        }
                    }
                    // one offer per wave per 64 iterations, by its first eligible lane (an offer
                    // walks the lane's lists: the wave waits for it)
                    const bool elig = !stop && !(frs & 5u) && n_aln == 0 && !C_OVF(ctl) && n_entries > 1 &&
                                      n_entries <= (int)FR_WALK && ps >= a.fr_budget && (fr_tick & 63u) == 0u;
                    const uint64_t em = __ballot(elig);
                    if (elig && lane == __ffsll((unsigned long long)em) - 1) {
                        const unsigned long long wt = __hip_atomic_load(&r->fr_c[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned long long rs = __hip_atomic_load(&r->fr_c[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned long long tk = __hip_atomic_load(&r->fr_c[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (wt > rs - tk + a.fr_demand) {     // more lanes wait than chunks do
                            if (!fr_offer()) frs |= 4u;
                            else if (frs & 2u) stop = true;      // a helper hands its rest on and ends
                            else { frs |= 1u; fr_p0 = st_p; fr_q0 = st_q; }
                        }
                    }
                    if (stop) { SET_PH(ctl, PH_END); continue; }
                }
            }
            if (C_VT(ctl)) {
                DC(3);
                ctl &= ~(1u << 6);                                        // e already holds it
            } else {
                DC(4);
                // pop the head of the lowest non-empty bucket
                const int b = mask.lowest();
                const uint32_t slot = HEAD(b);
                e = ent_load<IT>(a.pool, pbase, slot);
                const uint32_t nx = NXT(slot);
                if (nx == NIL) mask.reset(b);
                else HEAD(b) = (LT)nx;
                if (HUGE) { NXT(slot) = (LT)free_head; free_head = slot; }
            }
            --n_entries;
            ++st_p;
            const uint32_t m = e.w;
            if (!(R_MODE & MODE_NONSTOP) && SCORE(M_MM(m), M_GO(m), M_GE(m)) > best_score + S_MM) {
                SET_PH(ctl, PH_END);
                continue;
            }
            const int em = m_of(m);
            if (em < 0) { DC(18); continue; }
            const int ei = M_I(m);
            if (ei > 0 && em < (int)(wbg(ei - 1) & F::BIDM)) { DC(18); continue; }
            if (ei == 0) {
                DC(20);
                if (!on_hit(e.x, e.y, e.z, e.z + (e.y - e.x)) && !C_OVF(ctl)) SET_PH(ctl, PH_END);
                continue;
            }
            if (em == 0 && (M_ST(m) == ST_M || (R_MODE & MODE_GAPE) || M_GE(m) == R_MAXGE)) {
                ik = e.x; il = e.y; aux = e.z + (e.y - e.x); pos = (uint32_t)(ei - 1);   // bwt_match_exact
                SET_PH(ctl, PH_EXACT);
                continue;
            }
            req = 1; rp1 = e.x; rp2 = e.y + 1u;
            if constexpr (F::NIB) cur_c = getc(ei - 1);                  // the expansion's base (D)
            SET_PH(ctl, PH_EXPAND);
        } while (0);

#ifdef HSA_DIAG
        TMARK(1);
#endif
        // ---------------- (C) the rank step
        IT oa[4], ob[4];
#ifdef HSA_DIAG
        {
            const uint64_t rq = __ballot(req);
            if (lane == 0) dc[6] += (uint32_t)__popcll(rq);
            const uint32_t ph0 = C_PH(ctl);
            if (req) DC(ph0 == PH_EXACT ? 1 : 2);
            if (req && rp2 == rp1 + 1u) DC(ph0 == PH_EXACT ? 16 : 17);
        }
#endif
        uint32_t two = 0;
#ifdef HSA_DIAG
        rd_steps += req == 1 ? 1u : 0u;
#endif
        if (req == 1) {
            two = occ_pair(Ix<IT>::fwd(a), rp1, rp2, oa, ob) - 1u;
            st_q += 2u; st_b += 1u + two;
        }

#ifdef HSA_DIAG
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        TMARK(2);
#endif
        // ---------------- (D) apply
        const uint32_t ph = C_PH(ctl);
        if (F::NIB && req == 1 && ph == PH_EXACT && cur_c > 3) {
            st_q -= 2u; st_b -= 1u + two;                                // not a step (2BWT-Interface.c:377)
            SET_PH(ctl, PH_POP);
        } else if (req && ph == PH_EXACT) {
            // BWTSARangeBackward_Bidirection (2BWT-Interface.c:135-170), one character
            const uint32_t c = F::NIB ? cur_c : getc((int)pos);
            IT oc = 0;
#pragma unroll
            for (uint32_t d = 1; d < 4; ++d) oc += d > c ? ob[d] - oa[d] : (IT)0;
            const IT cc = pick4(CC, c);
            ik = cc + pick4(oa, c) + 1u;
            il = cc + pick4(ob, c);
            aux -= oc;                                                   // rev_l
            if (ik > il) {
                SET_PH(ctl, PH_POP);                                     // no match: continue (bwtgap.c:185)
            } else if (pos-- == 0) {
                // write-back guard of bwt_match_exact (2BWT-Interface.c:383-386)
                const IT rk = aux - (il - ik), erl = e.z + (e.y - e.x);
                const IT hk = e.x ? ik : (IT)0, hl = e.y ? il : (IT)0, hrk = e.z ? rk : (IT)0, hrl = erl ? aux : (IT)0;
                SET_PH(ctl, PH_POP);
                if (!on_hit(hk, hl, hrk, hrl) && !C_OVF(ctl)) SET_PH(ctl, PH_END);
            }
        } else if (req && ph == PH_EXPAND) {
            // children of the bidirectional step (2BWT-Interface.c:235-272), in place:
            // oa -> k, ob -> l of child c; srk = rev_k
            const uint32_t m = e.w;
            const IT ek = e.x, el = e.y, erk = e.z, erl = erk + (el - ek);
            const int i = M_I(m) - 1;                                    // --i (bwtgap.c:245)
            const int est = M_ST(m), emm = M_MM(m), ego = M_GO(m), ege = M_GE(m);
            const int em = m_of(m);
            const int len = C_LEN(ctl);
            IT srk[4];
            uint32_t ne = 0;                                             // children that occur
            {
                IT oc = 0;
#pragma unroll
                for (int c = 3; c >= 0; --c) {
                    const IT d = ob[c] - oa[c];
                    oa[c] = CC[c] + oa[c] + 1u;
                    ob[c] = CC[c] + ob[c];
                    srk[c] = (erl - oc) - (ob[c] - oa[c]);
                    oc += d;
                }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) ne |= (oa[c] <= ob[c] ? 1u : 0u) << c;
            int allow_diff = 1, allow_M = 1;
            if (i > 0) {
                // width[i-1].bid, width[i].bid and w[i-1] == w[i] (bwtgap.c:256-258)
                const uint32_t w1 = wbg(i - 1), w0 = wbg(i);
                const int b1 = (int)(w1 & F::BIDM), b0 = (int)(w0 & F::BIDM);
                if (b1 > em - 1) allow_diff = 0;
                else if (b1 == em - 1 && b0 == em - 1 && (w1 & F::EQ)) allow_M = 0;
                const int ii = i - (len - C_SLEN(ctl));
                if (C_SEED(ctl) && ii > 0) {
                    int ems = RG(max_seed_diff) - (emm + ego);
                    if (R_MODE & MODE_GAPE) ems -= ege;
                    // width_seed aliased to width_back (bwtgap.c:809): the same LDS row
                    const uint32_t s1 = C_ALIAS(ctl) ? wbg(ii - 1) : wsg(ii - 1);
                    const uint32_t s0 = C_ALIAS(ctl) ? wbg(ii) : wsg(ii);
                    const int c1 = (int)(s1 & F::BIDM), c0 = (int)(s0 & F::BIDM);
                    if (c1 > ems - 1) allow_diff = 0;
                    else if (c1 == ems - 1 && c0 == ems - 1 && (s1 & F::EQ)) allow_M = 0;
                }
            }
            // The pushes of bwtgap.c:267-325 as a candidate mask in push order:
            // bit 0 insertion, bits 1-4 deletion with child j = bit-1, bits 5-8
            // match/mismatch with child (seq[i] + bit-4) & 3.  All but the last go to the
            // pool in order; the last becomes the virtual top when it is the next pop.
            const uint32_t sc = F::NIB ? cur_c : getc(i);
            // (as selects over every case: nested ifs here were divergent branches)
            uint32_t cand = 0;
            if constexpr (GAPS) {
                const int ies = RG(indel_end_skip);
                const int tmp = (R_MODE & MODE_LOGGAP) ? int_log2((uint32_t)(ege + ego)) / 2 + 1 : ego + ege;
                const bool ok = (allow_diff != 0) & ((R_MAXGO > 0) | (ego > 0)) & (i >= ies + tmp) & (len - i >= ies + tmp);
                const IT occ = el - ek + 1u;
                const uint32_t c_m = ego < R_MAXGO ? (1u | ne << 1) : 0u;
                const uint32_t c_i = ege < R_MAXGE ? 1u : 0u;
                const bool d_ok = (ege < R_MAXGE) & ((ege + ego < max_diff) | (occ < (IT)RG(max_del_occ)));
                const uint32_t c_d = d_ok ? ne << 1 : 0u;
                const uint32_t c_g = est == ST_M ? c_m : est == ST_I ? c_i : c_d;
                cand = ok ? c_g : 0u;
            }
            {
                uint32_t c_mm = 0;
#pragma unroll
                for (int j = 1; j <= 4; ++j) {
                    const uint32_t c = (sc + (uint32_t)j) & 3u;
                    c_mm |= ((ne >> c) & 1u) << (4 + j);
                }
                const uint32_t c_eq = sc < 4 ? ((ne >> (sc & 3u)) & 1u) << 8 : 0u;   // == bit 8: c = sc, no mismatch
                cand |= (allow_diff & allow_M) ? c_mm : c_eq;
            }
            // entry of candidate bit b
            auto entry = [&](uint32_t b) -> E {
                const bool ins = GAPS && b == 0, del = GAPS && b >= 1 && b <= 4;
                const uint32_t c = del ? b - 1u : (sc + b - 4u) & 3u;
                const uint32_t is_mm = (b != 8u || sc > 3) ? 1u : 0u;
                IT k = pick4(oa, c), l = pick4(ob, c), rk = pick4(srk, c);
                uint32_t meta;
                if (GAPS && (ins || del)) {
                    if (ins) { k = ek; l = el; rk = erk; }
                    const uint32_t go = (uint32_t)ego + (est == ST_M), ge = (uint32_t)ege + (est != ST_M);
                    meta = meta_pack((uint32_t)(del ? i + 1 : i), ins ? ST_I : ST_D, 1u, (uint32_t)emm, go, ge);
                } else {
                    meta = meta_pack((uint32_t)i, ST_M, is_mm, (uint32_t)emm + is_mm, (uint32_t)ego, (uint32_t)ege);
                }
                return E{k, l, rk, meta};
            };
#ifdef HSA_DIAG
            // pushes whose pop would be pruned under the current max_diff and bids
            auto doomed = [&](uint32_t mw) {
                const int em2 = m_of(mw), i2 = M_I(mw);
                return em2 < 0 || (i2 > 0 && em2 < (int)(wbg(i2 - 1) & F::BIDM));
            };
#endif
            if (cand) {
                const uint32_t last = 31u - (uint32_t)__clz(cand);
                n_entries += __popc(cand);
                uint32_t rest = cand & ~(1u << last);
                if constexpr (HUGE) {
                    for (; rest; rest &= rest - 1u) {
                        const E v = entry((uint32_t)__ffs(rest) - 1u);
#ifdef HSA_DIAG
                        if (doomed(v.w)) DC(19);
#endif
                        flush(v, bucket_of(v.w));
                    }
                } else if (rest) {
                    // Every candidate but the last, in push order (gap_push, bwtgap.c:46-75),
                    // with each group's meta word and bucket computed once: the insertion
                    // and the deletions share one score, the mismatches another, the bit-8
                    // match child has the parent's.  The groups' bucket heads are kept in
                    // registers across the loop (equal buckets updated together, so the
                    // links are flush()'s) and written back once: the divergent loop does
                    // two stores per candidate and no LDS round trip.
                    const uint32_t g_go = (uint32_t)ego + (est == ST_M), g_ge = (uint32_t)ege + (est != ST_M);
                    const uint32_t mI = meta_pack((uint32_t)i, ST_I, 1u, (uint32_t)emm, g_go, g_ge);
                    const uint32_t mD = meta_pack((uint32_t)(i + 1), ST_D, 1u, (uint32_t)emm, g_go, g_ge);
                    const uint32_t mM = meta_pack((uint32_t)i, ST_M, 1u, (uint32_t)emm + 1u, (uint32_t)ego, (uint32_t)ege);
                    const uint32_t mP = meta_pack((uint32_t)i, ST_M, 0u, (uint32_t)emm, (uint32_t)ego, (uint32_t)ege);
                    const int bG = GAPS ? bucket_of(mI) : -1, bM = bucket_of(mM), bP = bucket_of(mP);
                    auto head0 = [&](int b) -> uint32_t {
                        return b >= 0 && (uint32_t)b < a.nb && mask.test(b) ? (uint32_t)HEAD(b) : NIL;
                    };
                    const uint32_t hG0 = GAPS ? head0(bG) : NIL, hM0 = head0(bM), hP0 = head0(bP);
                    uint32_t hG = hG0, hM = hM0, hP = hP0;
                    for (; rest; rest &= rest - 1u) {
                        const uint32_t b = (uint32_t)__ffs(rest) - 1u;
                        const bool ins = GAPS && b == 0, gap = GAPS && b <= 4u;
                        const bool mt = b == 8u && sc < 4;               // the match child
                        const uint32_t c = gap ? b - 1u : (sc + b - 4u) & 3u;
                        IT k = pick4(oa, c), l = pick4(ob, c), rk = pick4(srk, c);
                        if (ins) { k = ek; l = el; rk = erk; }
                        const uint32_t meta = ins ? mI : gap ? mD : mt ? mP : mM;
                        const int bk = gap ? bG : mt ? bP : bM;
#ifdef HSA_DIAG
                        if (doomed(meta)) DC(19);
#endif
                        if ((uint32_t)bk >= a.nb || pool_top >= a.pcap) { ctl |= 1u << 8; continue; }
                        const uint32_t slot = pool_top++;
                        DC(8);
                        ent_store<IT>(a.pool, pbase, slot, E{k, l, rk, meta});
                        NXT(slot) = (LT)(bk == bG ? hG : bk == bM ? hM : hP);
                        hG = bk == bG ? slot : hG;
                        hM = bk == bM ? slot : hM;
                        hP = bk == bP ? slot : hP;
                    }
                    if (GAPS && hG != hG0) { HEAD(bG) = (LT)hG; mask.set(bG); }
                    if (hM != hM0) { HEAD(bM) = (LT)hM; mask.set(bM); }
                    if (hP != hP0) { HEAD(bP) = (LT)hP; mask.set(bP); }
                }
                const E v = entry(last);
#ifdef HSA_DIAG
                if (doomed(v.w)) DC(19);
#endif
                const int bk = bucket_of(v.w);
                if (bk <= mask.lowest()) { e = v; ctl |= 1u << 6; }
                else flush(v, bk);
            }
            SET_PH(ctl, PH_POP);
        }
#ifdef HSA_DIAG
        TMARK(3);
#endif
    }

#ifdef HSA_DIAG
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        g_diag[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memtime();
        g_diag[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < 18; ++i)
        if (i < 9 || i > 12) atomicAdd(&g_dctr[i], (unsigned long long)dc[i]);
    for (int i = 18; i < 21; ++i) atomicAdd(&g_dctr[i], (unsigned long long)dc[i]);
    if (lane == 0)
        for (int i = 0; i < 4; ++i) atomicAdd(&g_dctr[9 + i], (unsigned long long)tsec[i]);
#endif
    // statistics
    if constexpr (FRH) {
        if (a.fr_budget) {
            unsigned long long hs = st_hs, hq = st_hq;
            for (int d = 32; d >= 1; d >>= 1) { hs += __shfl_xor(hs, d); hq += __shfl_xor(hq, d); }
            if (lane == 0) { atomicAdd(&a.fr_c[6], hs); atomicAdd(&a.fr_c[8], hq); }
        }
    }
    atomicAdd(&a.ctr[2], (unsigned long long)st_q);
    atomicAdd(&a.ctr[3], (unsigned long long)st_b);
    atomicAdd(&a.ctr[4], (unsigned long long)st_p);
    if (st_wq) {
        atomicAdd(&a.ctr[2], (unsigned long long)st_wq);
        atomicAdd(&a.ctr[7], (unsigned long long)st_wq);
        atomicAdd(&a.ctr[14], (unsigned long long)st_wq);
    }
#undef HEAD
#undef WB
#undef WS
#undef NXT
#undef HB
#undef RG
#undef S_MM
#undef S_GO
#undef S_GE
#undef R_MODE
#undef R_MAXGO
#undef R_MAXGE
#undef SCORE
}



#include "hsa_search_any.h"

// ---------------------------------------------------------------- host helpers (both TUs)
// What any search accepts (k_search_any's bounds); fast_regimes: what k_search's layouts hold.
static int check_regimes(const hsa_regime_t *rg, int n)
{
    for (int r = 0; r < n; ++r) {
        const hsa_regime_t &R = rg[r];
        if (R.s_mm < 0 || R.s_gapo < 0 || R.s_gape < 0) { hsa_set_error("negative penalty"); return HSA_E_ARG; }
        if (R.n_stacks <= 0 || R.n_stacks > ANY_MAX_STACKS) {
            hsa_set_error("n_stacks %d outside 1..%d", R.n_stacks, ANY_MAX_STACKS);
            return HSA_E_ARG;
        }
        if (R.max_gapo < 0 || R.max_gape < 0) { hsa_set_error("max_gapo/max_gape negative"); return HSA_E_ARG; }
        if (R.max_diff < -1) { hsa_set_error("max_diff out of range"); return HSA_E_ARG; }
    }
    return 0;
}

// Dense bucket numbering of the scores a search of this regime can push
// (bwtgap.c:46-75): n_mm <= max_diff+1, n_gapo <= min(max_gapo, max_diff), n_gape > 0
// only after a gap open.  Returns the bucket count.
static int bucket_map(const hsa_regime_t &R, uint8_t map[MAXS])
{
    bool used[MAXS] = {false};
    const int md = R.max_diff < 0 ? 0 : R.max_diff;
    const int go_max = R.max_gapo < md ? R.max_gapo : md;
    for (int mm = 0; mm <= md + 1; ++mm)
        for (int go = 0; go <= go_max; ++go)
            for (int ge = 0; ge <= (go > 0 ? R.max_gape : 0); ++ge) {
                const int s = mm * R.s_mm + go * R.s_gapo + ge * R.s_gape;
                if (s >= 0 && s < MAXS && s < R.n_stacks) used[s] = true;
            }
    int k = 0;
    for (int s = 0; s < MAXS; ++s) map[s] = used[s] && k < 0xFF ? (uint8_t)k++ : (uint8_t)0xFF;
    return k;
}

// Regimes whose every bound fits k_search's layouts: the entry meta word (n_gapo 4
// bits, n_gape 8, n_mm 7), the score table (MAXS), the bucket mask (MAXB reachable
// scores) and the 16-bit pruning elements (bids compared with bounds <= 254).  Other
// regimes run k_search_any.
static bool fast_regimes(const hsa_regime_t *rg, int n)
{
    if (getenv("HSA_FORCE_ANY")) return false;       // tests: every search through k_search_any
    for (int r = 0; r < n; ++r) {
        const hsa_regime_t &R = rg[r];
        if (R.max_gapo > 14 || R.max_gape > 254 || R.max_diff > 125 || R.max_seed_diff > 254 || R.n_stacks > MAXS)
            return false;
        uint8_t map[MAXS];
        if (bucket_map(R, map) > MAXB) return false;
    }
    return true;
}

#define FAST_MAX_LEN 1023u       // k_search: 10-bit read positions (meta word, control word)

// The dense bucket of a score is simply its n_mm when no gap opens exist and every
// reachable mismatch count has its own score (k_search skips the table then).
static bool mm_buckets(const hsa_regime_t *rg, int n, const uint8_t *bmap)
{
    for (int r = 0; r < n; ++r) {
        const hsa_regime_t &R = rg[r];
        if (R.max_gapo != 0 || R.s_mm <= 0) return false;
        const int md = R.max_diff < 0 ? 0 : R.max_diff;
        for (int mm = 0; mm <= md + 1; ++mm) {
            const int sc = mm * R.s_mm;
            if (sc >= MAXS || bmap[r * MAXS + sc] != mm) return false;
        }
    }
    return true;
}

struct LaunchPlan {
    size_t lanes, blocks;
    uint32_t nt;                     // lanes per workgroup of k_search (256 or 64)
    uint32_t pcap, hcap, nb;
    bool gaps, wide;                 // gap opens possible; 16-bit pruning elements (WFmt)
    bool nib;                        // 4-bit pruning elements in LDS (WFmt<WNib>)
    uint32_t off_heads, off_wb, off_ws;
    uint32_t nib_wb, nib_ws;         // 4-bit rows: LDS words per lane (SearchArgs)
    size_t lds;
    bool huge;                       // PASS_HUGE: 32-bit links, reused slots
    uint32_t ntab;                   // score table entries per regime in LDS
    size_t resident;                 // lanes resident on the chip (every CU full)
    size_t res_lanes = 0;            // lanes the scratch is reserved for (BIG: all its lanes)
};

// The capacity passes of one search: MAIN (every read), BIG (the reads that overflowed
// their main-pass lane: 65 535 pool slots, 16 384 hits), HUGE (the reads that overflowed
// BIG: reused slots up to max_entries + 16 live entries, 262 144 hits).
enum { PASS_MAIN = 0, PASS_BIG = 1, PASS_HUGE = 2 };

static int plan_launch(hsa_index *ix, int n_jobs, int max_len, int max_seed, int nb, bool gaps, bool wide, int mode,
                       LaunchPlan &P, int max_entries = 0, uint32_t ent_bytes = 16, bool nib_ok = false)
{
    const bool big = mode == PASS_BIG;
    P.huge = mode == PASS_HUGE;
    P.ntab = (uint32_t)ix->staged_ntab;
    P.nb = (uint32_t)nb;
    P.gaps = gaps;
    P.wide = wide;
    const uint32_t esz = wide ? 2u : 1u;
    P.nib = false;
    // Resident workgroups per CU, from gfx950's own limits: 160 KiB of LDS per CU, at
    // most 16 waves (__launch_bounds__(NT, 4) caps VGPRs at 4 waves per SIMD).  The
    // per-lane LDS (bucket heads, pruning rows) decides between 256-lane workgroups
    // and 64-lane ones, which pack the CU's LDS more finely: -n 4 -o 1 has 39 buckets
    // and ~220 B per lane, i.e. 2 workgroups of 256 (8 waves) but 11 of 64 (11 waves).
    // (hipOccupancyMaxActiveBlocksPerMultiprocessor is not used: depending on which
    // HIP runtime the process loaded first it assumed 64 KiB of LDS and halved the
    // grid -- measured 512 instead of 1024 workgroups, 1.5x slower.)
    auto layout = [&](uint32_t nt) {
        const uint32_t epw = P.nib ? 8u : 4u / esz;      // elements per LDS word (WFmt::EPW)
        P.nt = nt;
        P.off_heads = 2 * P.ntab + 128;   // score tables, then the two regimes
        P.off_wb = P.off_heads + (uint32_t)nb * nt * (P.huge ? 4u : 2u);
        // k_search reads elements 0 .. len - 1 of a row (pops of position i read i - 1,
        // expansions i - 1 and i < len; seed rows ii - 1 and ii < seed_len): the 4-bit
        // rows keep just those, which takes config 5's 64-lane workgroups from 15 to 16
        // per CU; the 8-bit rows keep element len too (the LDS-DMA copies whole words)
        P.nib_wb = ((uint32_t)max_len + 7u) / 8u;
        P.nib_ws = ((uint32_t)max_seed + 7u) / 8u;
        const uint32_t wbw = P.nib ? P.nib_wb : (uint32_t)max_len / epw + 1u;
        const uint32_t wsw = P.nib ? P.nib_ws : (uint32_t)max_seed / epw + 1u;
        P.off_ws = P.off_wb + wbw * nt * 4u;
        P.lds = ((size_t)P.off_ws + (size_t)wsw * nt * 4u + 15) / 16 * 16;
        int per_cu = (int)((160u * 1024u) / P.lds);
        const int cap = 4 * HSA_WAVES_SIMD / (int)(nt / 64);  // 16 waves per CU
        const int want = g_waves_per_cu / (int)(nt / 64);
        if (per_cu > cap) per_cu = cap;
        if (per_cu > want) per_cu = want > 0 ? want : 1;
        return per_cu;
    };
    static const int force256 = getenv("HSA_WG256") != nullptr;   // A/B runs only
    auto best = [&]() {
        int per_cu = layout(P.huge ? 64 : 256);
        if (per_cu < 4 && !force256 && !P.huge) {
            const int p64 = layout(64);
            if (p64 > per_cu * 4) per_cu = p64;
            else per_cu = layout(256);
        }
        return per_cu;
    };
    int per_cu = best();
    // long reads: 4-bit elements when the 8-bit rows leave the CU short of 16 waves, in
    // ungapped searches, which are latency-bound: config 5's k_search 45.6 -> 38.4 ms.
    // Gapped ones are issue-bound and lose more to the unpacking and the base loads
    // than they gain in waves (config 4: 1 988 -> 2 147 ms; config 3: equal).
    // HSA_WFMT=nib forces them where exact, =byte keeps 8-bit (tests and A/B runs).
    const char *wf = getenv("HSA_WFMT");
    const bool force_nib = wf && !strcmp(wf, "nib"), no_nib = wf && !strcmp(wf, "byte");
    if (nib_ok && !wide && !P.huge && !no_nib && (force_nib || (!gaps && per_cu * (int)(P.nt / 64) < 16))) {
        const int waves8 = per_cu * (int)(P.nt / 64);
        const LaunchPlan keep = P;
        P.nib = true;
        const int per_nib = best();
        if (!force_nib && per_nib * (int)(P.nt / 64) <= waves8) { P = keep; }
        else per_cu = per_nib;
    }
    if (P.lds > 160 * 1024) { hsa_set_error("reads too long for the LDS budget (%zu bytes)", P.lds); return HSA_E_ARG; }
    if (per_cu < 1) { hsa_set_error("search kernel does not fit (LDS %zu)", P.lds); return HSA_E_ARG; }
    const uint32_t NTB = P.nt;
    size_t blocks = (size_t)ix->n_cu * per_cu;
    P.resident = blocks * NTB;
    size_t need_blocks = ((size_t)n_jobs + NTB - 1) / NTB;
    if (P.huge) {
        blocks = 1;                                          // 64 lanes: a handful of reads
    } else if (big) {
        static const size_t big_lanes = getenv("HSA_BIG_LANES") ? strtoull(getenv("HSA_BIG_LANES"), nullptr, 10) : 4096;
        const size_t big_blocks = big_lanes / NTB > 0 ? big_lanes / NTB : 1;
        blocks = need_blocks < big_blocks ? need_blocks : big_blocks;
        // the BIG pass's scratch is reserved for all its lanes whatever the pass's size:
        // the attach-time warm-up then allocates it (7.3 GB at the default shape) instead
        // of a process's first full batch
        P.res_lanes = big_blocks * NTB;
    } else if (need_blocks < blocks) {
        blocks = need_blocks;
    }
    if (blocks < 1) blocks = 1;
    P.blocks = blocks;
    P.lanes = blocks * NTB;
    if (getenv("HSA_VERBOSE")) {                   // read per plan: tests switch it on mid-process
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_search<1, true, uint8_t, 256>, 256, P.lds);
        fprintf(stderr, "[hsa] launch: %d CUs x %d workgroups of %u lanes (runtime occupancy query says %d), "
                "LDS %zu B, %zu workgroups, %d buckets%s\n", ix->n_cu, per_cu, P.nt, occ, P.lds, blocks, nb,
                P.nib ? ", 4-bit rows" : "");
    }
    // pool slots are not reused within a search: gapped searches push many more.  A
    // deeper main-pass pool keeps the long gapped searches inside the main pass, where
    // their tails overlap other lanes' work, instead of the serial overflow re-run:
    // config 4 (150 bp, -o 1) 2.36 -> 2.07 s per 1M reads at 32768 (49152: same)
    static const int pool_env = getenv("HSA_POOL_ENTRIES") ? atoi(getenv("HSA_POOL_ENTRIES")) : 0;   // A/B runs
    const int pool_main = g_pool_entries ? g_pool_entries : pool_env > 0 && pool_env <= 65535 ? pool_env : 0;
    // gapped reads of up to 128 bases: 16 384 (config 3 at 32 768: 106 GB of scratch per
    // handle; at 16 384 53 GB and k_search 284.9 -> 283.7 ms, profiles/r05_pool16k_ab.log);
    // longer gapped reads keep 32 768 (config 4 at 8 192: 32 s against 1.2 s)
    P.pcap = big ? 65535u : (uint32_t)(pool_main ? pool_main : (gaps ? (max_len <= 128 ? 16384 : 32768) : 8192));
    // searches of at most 32 bases (the splice path's 12-mer anchors, which run on every
    // resident lane) keep 8 192 entries with gap opens too: 155 -> 39 GB of scratch per
    // handle at config 4, the anchors' time unchanged (profiles/r05_pool_short_ab.log);
    // HSA_POOL_SHORT=n sets it (0: the regime's default)
    static const int pool_short = getenv("HSA_POOL_SHORT") ? atoi(getenv("HSA_POOL_SHORT")) : 8192;
    if (!big && !pool_main && max_len <= 32 && pool_short > 0 && pool_short <= 65535) P.pcap = (uint32_t)pool_short;
    P.hcap = big ? 16384u : (uint32_t)g_hit_cap;
    if (P.huge) {
        // live entries never exceed max_entries + 9 (bwtgap.c:150-151); the pool is
        // capped at 4 Mi entries per lane (80 MB), beyond which a read stays unfinished
        const uint64_t want = (uint64_t)(max_entries > 0 ? max_entries : 0) + 16u;
        P.pcap = (uint32_t)(want < (4ull << 20) ? want : (4ull << 20));
        P.hcap = 262144u;
    } else if (ent_bytes > 16 && !big) {
        // 64-bit entries are 32 bytes: the main pass's pools stay within 64 GB of HBM
        // (next to an index of up to ~2 x 16 GB for a 15 Gbp text); reads that need
        // more go to the big and huge passes as usual
        const size_t budget = (size_t)64 << 30;
        if (P.lanes * P.pcap * ent_bytes > budget) {
            const size_t p = budget / (P.lanes * ent_bytes);
            P.pcap = (uint32_t)(p < 1024 ? 1024 : p);
        }
    }
    return 0;
}

template <typename WT, int NT, typename IT>
static void launch_search_nt(const LaunchPlan &P, const SearchArgs &A, hipStream_t st)
{
    const dim3 g((unsigned)P.blocks), b(NT);
    if (P.nb <= 32) {
        if (P.gaps) hipLaunchKernelGGL((k_search<0, true, WT, NT, false, IT>), g, b, P.lds, st, A);
        else hipLaunchKernelGGL((k_search<0, false, WT, NT, false, IT>), g, b, P.lds, st, A);
    } else if (P.nb <= 64) {
        if (P.gaps) hipLaunchKernelGGL((k_search<1, true, WT, NT, false, IT>), g, b, P.lds, st, A);
        else hipLaunchKernelGGL((k_search<1, false, WT, NT, false, IT>), g, b, P.lds, st, A);
    } else {
        if (P.gaps) hipLaunchKernelGGL((k_search<2, true, WT, NT, false, IT>), g, b, P.lds, st, A);
        else hipLaunchKernelGGL((k_search<2, false, WT, NT, false, IT>), g, b, P.lds, st, A);
    }
}

template <typename WT, typename IT>
static void launch_search(const LaunchPlan &P, const SearchArgs &A, hipStream_t st)
{
    if constexpr (!std::is_same<WT, WNib>::value) {
        if (P.nib) {                                 // never a HUGE pass (plan_launch)
            if (P.nt == 64) launch_search_nt<WNib, 64, IT>(P, A, st);
            else launch_search_nt<WNib, 256, IT>(P, A, st);
            return;
        }
    }
    if (P.huge) {
        const dim3 g((unsigned)P.blocks), b(64);
        if (P.gaps) hipLaunchKernelGGL((k_search<2, true, WT, 64, true, IT>), g, b, P.lds, st, A);
        else hipLaunchKernelGGL((k_search<2, false, WT, 64, true, IT>), g, b, P.lds, st, A);
        return;
    }
    if (P.nt == 64) launch_search_nt<WT, 64, IT>(P, A, st);
    else launch_search_nt<WT, 256, IT>(P, A, st);
}

// One search pass over jobs (or a job_list subset) with device pointers: k_widths
// fills the width rows of every (read, strand), then k_search runs the reads.
// caller-width mode of a pass (hsa_match_gap_batch)
struct MgPass {
    const hsa_mg_job_t *d_mg;
    int32_t *d_cw;
};

template <typename IT = uint32_t>
static SearchArgs pass_args(hsa_index *ix, const LaunchPlan &P, SearchScratch &S, const hsa_regime_t *d_regimes,
                            const uint8_t *d_bmap, const hsa_job_t *d_jobs, const int32_t *d_list, int n, int max_len,
                            int max_seed, const uint8_t *d_codes, int32_t *d_n, uint32_t *d_fl, uint64_t *d_ho,
                            uint32_t *d_hits, uint64_t hit_cap, unsigned long long *d_ctr, const MgPass *mg)
{
    constexpr size_t WGB = sizeof(IT);       // bytes per full w value (wg rows)
    const uint32_t esz = P.wide ? 2u : 1u;
    const uint32_t rb = (((uint32_t)max_len + 1u) * esz + 3u) & ~3u, rs = (((uint32_t)max_seed + 1u) * esz + 3u) & ~3u;
    const uint32_t rg = (uint32_t)max_len + 1u;
    const size_t rows = ((size_t)n + 63) / 64 * 64 * 2;     // two 64-row-aligned planes (lazy widths)
    uint8_t *wr = (uint8_t *)ix->d_wrows;
    SearchArgs A;
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T;
    memcpy(A.C, ix->C, sizeof A.C);
    A.fwd64 = hsa_rank_dir64(ix, 0);
    A.rev64 = hsa_rank_dir64(ix, 1);
    A.T64 = ix->T64;
    memcpy(A.C64, ix->C64, sizeof A.C64);
    A.regimes = d_regimes; A.bmap = d_bmap; A.jobs = d_jobs; A.job_list = d_list; A.n_jobs = n; A.codes = d_codes;
    A.n_aln = d_n; A.flags = d_fl; A.hit_off = d_ho; A.hits = d_hits; A.hit_cap = hit_cap; A.ctr = d_ctr;
    A.wb = wr; A.ws = wr + rows * rb; A.wg = reinterpret_cast<uint32_t *>(wr + rows * (rb + rs));
    A.rb = rb; A.rs = rs; A.rg = rg;
    A.pool = S.pool; A.nxt = S.nxt; A.hbuf = S.hbuf;
    A.pcap = P.pcap; A.hcap = P.hcap;        // the planned capacities (the scratch may be larger)
    A.nb = P.nb; A.off_heads = P.off_heads; A.off_wb = P.off_wb; A.off_ws = P.off_ws;
    A.nib_wb = P.nib_wb; A.nib_ws = P.nib_ws;
    A.mm_buckets = ix->staged_mmb ? 1u : 0u;
    A.ntab = P.ntab;
    A.batch_k = (uint32_t)g_batch_k;
    A.batch_idle = (uint32_t)g_batch_idle;
    A.ovf_list = nullptr; A.n_dev = nullptr; A.qctr = 0; A.ovf_ctr = 8;
    A.split = 0; A.sp_n = nullptr; A.sp_off = nullptr; A.sp_q = nullptr; A.sp_p = nullptr;
    const char *te = getenv("HSA_TRIE");           // HSA_TRIE=0: rank steps only (A/B runs)
    const bool tr = ix->trie_depth > 0 && ix->trie_wide == (sizeof(IT) == 8) && !(te && atoi(te) == 0);
    A.ktw = tr ? ix->d_trie_w : nullptr;
    A.ktd = tr ? ix->trie_depth : 0u;
    A.wkey = nullptr; A.perm = nullptr; A.okey = 0;
    A.fwd_list = nullptr; A.fwd_n = nullptr; A.fwd_only = 0; A.rmap = nullptr;
    A.fr_budget = 0; A.fr_demand = 0; A.fr_cap = 0;
    A.fr_ent = nullptr; A.fr_tag = nullptr; A.fr_rq = nullptr; A.fr_st = nullptr; A.fr_q = nullptr; A.fr_p = nullptr; A.fr_c = nullptr;
    A.mg = mg ? mg->d_mg : nullptr;
    A.cw = mg ? mg->d_cw : nullptr;
    A.wbid = mg ? reinterpret_cast<int32_t *>(wr + rows * (rb + rs + WGB * (size_t)rg)) : nullptr;
    A.wq = reinterpret_cast<uint32_t *>(wr + rows * (rb + rs + WGB * (size_t)rg + (mg ? 4 * (size_t)rg : 0)));
    return A;
}

// Strand-split mode for the main pass of a small batch: each read's two strands on two
// lanes when both fit on the chip at once (HSA_SPLIT=0/1 forces it off/on).  A read's
// search chain halves (rc and fwd side by side); the fwd strand's work is speculative, so
// large batches, which fill every lane anyway, keep one read per lane.
// Helpers are opt-in (HSA_HELP=1): exact, but measured slower on the drop-in's 100 000-read
// calls ("Helpers")
static bool use_help()
{
    const char *e = getenv("HSA_HELP");
    return e && atoi(e) != 0;
}

// (helpers run in gapped 32-bit kernels only, k_search's FRH)
template <typename IT>
static bool help_kernel(const LaunchPlan &P) { return use_help() && HSA_HELPERS && P.gaps && sizeof(IT) == 4; }

static bool use_split(const LaunchPlan &P, int n, const unsigned long long *n_dev, const MgPass *mg, uint32_t qctr,
                      bool help)
{
    if (mg || n_dev || qctr != 0 || P.huge || n <= 0) return false;
    const char *e = getenv("HSA_SPLIT");
    if (e) return atoi(e) != 0;
    // with helpers, also batches of up to one read per resident lane: their tails are the
    // long strand searches the waiting lanes then share
    return (help ? (size_t)n : 2 * (size_t)n) <= P.resident;
}

// Helpers of a strand-split pass (SearchArgs::fr_*): the shared frontier and the per-item
// state in ix->d_help, zeroed on the pass's stream.  HSA_HELP=0: off; HSA_HELP_BUDGET pops
// before a strand may offer its entries (default 512); HSA_HELP_DEMAND waiting lanes beyond
// the unsearched chunks before it does (default: half the pass's lanes, so that only the
// strands still running when half the chip waits -- the launch's tail -- offer); HSA_HELP_CAP
// chunks of FR_CH entries (default 1 Mi: 512 MB).
// Off when a regime's max_entries does not exceed the pool: then the main pass's stack
// stays below the reference's max_entries break (bwtgap.c:150-151) whenever it completes,
// and a strand its helpers answer counts the reference's rank queries and pops.
template <typename IT>
static int help_args(hsa_index *ix, SearchArgs &A, size_t items, const LaunchPlan &P, hipStream_t st)
{
    if (!help_kernel<IT>(P) || ix->staged_min_entries <= (int)P.pcap + 16) return 0;
    auto env = [](const char *k, long d) { const char *v = getenv(k); return v ? atol(v) : d; };
    const long budget = env("HSA_HELP_BUDGET", 512), demand = env("HSA_HELP_DEMAND", (long)(P.lanes / 2));
    const long cap = env("HSA_HELP_CAP", 1l << 20);
    if (budget <= 0 || cap <= 0 || cap > (1l << 24) || demand < 0 || items >= (1u << 26)) return 0;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_st = 256, o_q = o_st + al(items * 4), o_p = o_q + al(items * 8), o_tag = o_p + al(items * 8);
    const size_t o_rq = o_tag + al((size_t)cap * 4);
    const size_t o_ent = o_rq + al((size_t)cap * 4), total = o_ent + (size_t)cap * FR_CH * FR_EW * 4;
    int rc = hsa_grow(&ix->d_help, &ix->d_help_cap, total);
    if (rc) return rc;
    char *d = (char *)ix->d_help;
    HSA_HIP(hipMemsetAsync(d, 0, o_ent, st));       // counters, item state and sums, tags, ready queue
    A.fr_budget = (uint32_t)budget; A.fr_demand = (uint32_t)demand; A.fr_cap = (uint32_t)cap;
    A.fr_c = (unsigned long long *)d;
    A.fr_st = (uint32_t *)(d + o_st);
    A.fr_q = (unsigned long long *)(d + o_q);
    A.fr_p = (unsigned long long *)(d + o_p);
    A.fr_tag = (uint32_t *)(d + o_tag);
    A.fr_rq = (uint32_t *)(d + o_rq);
    A.fr_ent = (uint32_t *)(d + o_ent);
    return 0;
}

// The pass's search scratch (per-lane pools, links, staged hits), sized to what the
// device can give: the pool per lane is the plan's capacity unless that would not fit in
// the free HBM (less a 2 GiB margin) or in HSA_SCRATCH_MB, in which case it is halved
// until it does (down to 512 entries), and again if the allocation itself fails.  A
// smaller pool changes no result: a read that outgrows its lane is re-run in the BIG and
// HUGE passes as before, so the cost is speed, never an error (the reference's capacity
// bound is max_entries, bwtgap.c:150-151, which the HUGE pass keeps).
static int scratch_fit(hsa_index *ix, SearchScratch &S, LaunchPlan &P, size_t EW)
{
    const size_t lb = P.huge ? 4 : 2, floor_cap = 512;
    auto pe_of = [&](uint32_t pc) { return (size_t)((pc + 31u) & ~31u) * EW; };
    const size_t rl = P.res_lanes > P.lanes ? P.res_lanes : P.lanes;
    auto bytes = [&](uint32_t pc) { return rl * (pe_of(pc) * (16 + lb) + (size_t)P.hcap * EW * 36); };
    const bool held = S.pool && lb == S.link_bytes && rl * pe_of(P.pcap) <= S.pool_entries &&
                      rl * (size_t)P.hcap * EW <= S.hit_entries;
    if (!held && !P.huge) {
        const char *cm = getenv("HSA_SCRATCH_MB");      // read per pass: tests set it mid-process
        const size_t cap_mb = cm ? strtoull(cm, nullptr, 10) : 0;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); fr = (size_t)-1 / 2; }
        fr += S.pool_entries * (16 + S.link_bytes) + S.hit_entries * 36;     // what the reservation frees first
        size_t avail = fr > ((size_t)2 << 30) ? fr - ((size_t)2 << 30) : 0;
        if (cap_mb && avail > (cap_mb << 20)) avail = cap_mb << 20;
        const uint32_t want = P.pcap;
        while (bytes(P.pcap) > avail && P.pcap > floor_cap) P.pcap = P.pcap / 2 > floor_cap ? P.pcap / 2 : floor_cap;
        if (P.pcap != want && getenv("HSA_VERBOSE"))
            fprintf(stderr, "[hsa] search scratch: pool %u -> %u entries per lane (%.1f GB for %zu lanes; %.1f GB "
                            "available)\n", want, P.pcap, bytes(P.pcap) / 1e9, P.lanes, avail / 1e9);
    }
    for (;;) {
        const int rc = hsa_scratch_reserve(S, rl, pe_of(P.pcap), (size_t)P.hcap * EW, lb);
        if (rc != HSA_E_MEM || P.huge || P.pcap <= floor_cap) return rc;
        P.pcap = P.pcap / 2 > floor_cap ? P.pcap / 2 : floor_cap;
        if (getenv("HSA_VERBOSE")) fprintf(stderr, "[hsa] search scratch: allocation failed, pool -> %u per lane\n", P.pcap);
    }
}

template <typename IT = uint32_t>
static int launch_pass(hsa_index *ix, const LaunchPlan &P0, SearchScratch &S, const hsa_regime_t *d_regimes,
                       const uint8_t *d_bmap, const hsa_job_t *d_jobs, const int32_t *d_list, int n, int max_len,
                       int max_seed, const uint8_t *d_codes, int32_t *d_n, uint32_t *d_fl, uint64_t *d_ho,
                       uint32_t *d_hits, uint64_t hit_cap, unsigned long long *d_ctr, hipStream_t st,
                       int32_t *ovf_list = nullptr, const unsigned long long *n_dev = nullptr, uint32_t qctr = 0,
                       const MgPass *mg = nullptr, uint32_t ovf_ctr = 8)
{
    const bool split = use_split(P0, n, n_dev, mg, qctr, help_kernel<IT>(P0));
    LaunchPlan P = P0;
    if (split) {                                        // lanes for 2 n items
        const size_t need = (2 * (size_t)n + P.nt - 1) / P.nt, cap = P.resident / P.nt;
        P.blocks = need < cap ? need : cap;
        P.lanes = P.blocks * P.nt;
    }
    // 64-bit intervals: two uint4 per pool entry, 10 staged words per hit (HitW)
    constexpr size_t EW = sizeof(IT) / 4;
    int rc = scratch_fit(ix, S, P, EW);
    if (rc) return rc;
    const uint32_t esz = P.wide ? 2u : 1u;
    const uint32_t rb = (((uint32_t)max_len + 1u) * esz + 3u) & ~3u, rs = (((uint32_t)max_seed + 1u) * esz + 3u) & ~3u;
    const uint32_t rg = (uint32_t)max_len + 1u;
    const size_t rows = ((size_t)n + 63) / 64 * 64 * 2;     // two 64-row-aligned planes (lazy widths)
    const size_t row_bytes = rb + rs + sizeof(IT) * (size_t)rg + (mg ? 4 * (size_t)rg : 0);   // + full bids (caller widths)
    // + wq (4 n), cost keys (2 n), order (4 n) and its 32 counters
    if ((rc = hsa_grow(&ix->d_wrows, &ix->d_wrows_cap, rows * row_bytes + 10 * (size_t)n + 1024))) return rc;
    if (mg) {
        if constexpr (sizeof(IT) != 4) {
            hsa_set_error("caller-width searches (bwt_match_gap) take 32-bit indexes");
            return HSA_E_ARG;
        } else {
            SearchArgs A = pass_args<IT>(ix, P, S, d_regimes, d_bmap, d_jobs, d_list, n, max_len, max_seed, d_codes, d_n,
                                         d_fl, d_ho, d_hits, hit_cap, d_ctr, mg);
            A.ovf_list = ovf_list; A.n_dev = n_dev; A.qctr = qctr; A.ovf_ctr = ovf_ctr;
            if (qctr == 0) HSA_HIP(hipMemsetAsync(d_ctr, 0, 16 * sizeof(unsigned long long), st));   // not on a re-run
            const unsigned nb = (unsigned)(((size_t)n + BLOCK - 1) / BLOCK);
            if (P.wide) hipLaunchKernelGGL(k_widths_import<uint16_t>, dim3(nb ? nb : 1), dim3(BLOCK), 0, st, A);
            else hipLaunchKernelGGL(k_widths_import<uint8_t>, dim3(nb ? nb : 1), dim3(BLOCK), 0, st, A);
            HSA_HIP(hipGetLastError());
            if (ix->ev_split) HSA_HIP(hipEventRecord(ix->ev_split, st));
            if (P.wide) launch_search<uint16_t, uint32_t>(P, A, st);
            else launch_search<uint8_t, uint32_t>(P, A, st);
            HSA_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_widths_export, dim3(nb ? nb : 1), dim3(BLOCK), 0, st, A);
            HSA_HIP(hipGetLastError());
            return 0;
        }
    }
    SearchArgs A = pass_args<IT>(ix, P, S, d_regimes, d_bmap, d_jobs, d_list, n, max_len, max_seed, d_codes, d_n, d_fl,
                                 d_ho, d_hits, hit_cap, d_ctr, nullptr);
    A.ovf_list = ovf_list; A.n_dev = n_dev; A.qctr = qctr; A.ovf_ctr = ovf_ctr;
    if (split) {
        const size_t m = 2 * (size_t)n, al = (m * 8 + 255) / 256 * 256;
        if ((rc = hsa_grow(&ix->d_split, &ix->d_split_cap, 3 * al))) return rc;
        char *d = (char *)ix->d_split;
        A.split = 1;
        A.sp_off = (uint64_t *)d;
        A.sp_n = (int32_t *)(d + al);
        A.sp_q = (uint32_t *)(d + al + al / 2);
        A.sp_p = (uint32_t *)(d + 2 * al);
        if (!P.huge && (rc = help_args<IT>(ix, A, m, P, st))) return rc;
    }
    if (qctr == 0) HSA_HIP(hipMemsetAsync(d_ctr, 0, 16 * sizeof(unsigned long long), st));   // not on a re-run
    // cost order: the main pass of a batch with more reads than the chip has lanes
    // (HSA_ORDER=0/1 forbids / forces it)
    const char *oe = getenv("HSA_ORDER");
    const bool order = !split && !n_dev && qctr == 0 && n > 0 &&
                       (oe ? atoi(oe) != 0 : (size_t)n > P.resident);
    uint32_t *d_oh = nullptr;
    if (order) {
        char *tail = (char *)A.wq + 4 * (size_t)n;
        A.wkey = (uint8_t *)tail;
        // the tail-length key: config 2 k_search 18.5-18.9 -> 17.9-18.0 ms, config 3 and 5 1-2 %
        // (profiles/r03_ab2_okey_*); HSA_ORDER_KEY=0: the final bid alone
        static const uint32_t okey = getenv("HSA_ORDER_KEY") ? (uint32_t)atoi(getenv("HSA_ORDER_KEY")) : 1u;
        A.okey = okey;
        const size_t ko = (2 * (size_t)n + 15) / 16 * 16;
        d_oh = (uint32_t *)(tail + ko);
        HSA_HIP(hipMemsetAsync(d_oh, 0, 32 * 4, st));
    }
    // lazy forward rows: the main pass of a batch searched one read per lane computes a
    // read's forward row only when its rc search cannot hit; the reads whose rc search
    // finds nothing without one get it in the forward pass below.  It pays for long reads
    // (config 5's 250 bp: k_widths 17.0 -> 15.7 ms); for 100 bp reads the second width
    // launch costs more than the rows it saves (5.25 -> 5.68 ms), so by default reads of
    // 200 bases or more (HSA_LAZY=0 / 1 forbids / forces it)
    const char *le = getenv("HSA_LAZY");
    const bool lazy = !split && !n_dev && qctr == 0 && n > 0 && (le ? atoi(le) != 0 : max_len >= 200);
    unsigned long long *d_fwd_n = nullptr;
    int32_t *d_list2 = nullptr;
    unsigned long long *d_n2 = nullptr;
    if (lazy) {
        // [count, count2 | forward-pass list (n) | list2 (n)]
        if ((rc = hsa_grow(&ix->d_fwd, &ix->d_fwd_cap, 512 + 12 * (size_t)n))) return rc;
        d_fwd_n = (unsigned long long *)ix->d_fwd;
        d_n2 = d_fwd_n + 1;
        HSA_HIP(hipMemsetAsync(d_fwd_n, 0, 16, st));
        A.fwd_n = d_fwd_n;
        A.fwd_list = (int32_t *)((char *)ix->d_fwd + 128);
        d_list2 = A.fwd_list + ((size_t)n + 31) / 32 * 32;
        A.rmap = d_list2 + ((size_t)n + 31) / 32 * 32;
    }
    if (lazy) {
        const unsigned rblocks = (unsigned)(((size_t)n + BLOCK - 1) / BLOCK);
        if (P.wide) {
            hipLaunchKernelGGL((k_widths_reads<uint16_t, IT>), dim3(rblocks), dim3(BLOCK), 0, st, A, 1u, d_list2, d_n2);
            hipLaunchKernelGGL((k_widths_reads<uint16_t, IT>), dim3(rblocks), dim3(BLOCK), 0, st, A, 3u, d_list2, d_n2);
        } else {
            hipLaunchKernelGGL((k_widths_reads<uint8_t, IT>), dim3(rblocks), dim3(BLOCK), 0, st, A, 1u, d_list2, d_n2);
            hipLaunchKernelGGL((k_widths_reads<uint8_t, IT>), dim3(rblocks), dim3(BLOCK), 0, st, A, 3u, d_list2, d_n2);
        }
    } else {
        size_t wblocks = ((size_t)n * 2 + BLOCK - 1) / BLOCK;
        if (wblocks < 1) wblocks = 1;
        if (P.wide) hipLaunchKernelGGL((k_widths<uint16_t, IT>), dim3((unsigned)wblocks), dim3(BLOCK), 0, st, A);
        else hipLaunchKernelGGL((k_widths<uint8_t, IT>), dim3((unsigned)wblocks), dim3(BLOCK), 0, st, A);
    }
    HSA_HIP(hipGetLastError());
    if (order) {
        int32_t *d_perm = (int32_t *)(d_oh + 32);
        const unsigned nb = (unsigned)(((size_t)n + BLOCK - 1) / BLOCK);
        hipLaunchKernelGGL(k_order_hist, dim3(nb), dim3(BLOCK), 0, st, A, d_oh);
        hipLaunchKernelGGL(k_order_scan, dim3(1), dim3(1), 0, st, d_oh);
        hipLaunchKernelGGL(k_order_scatter, dim3(nb), dim3(BLOCK), 0, st, A, d_oh, d_perm);
        HSA_HIP(hipGetLastError());
        A.perm = d_perm;
    }
    if (ix->ev_split && qctr == 0) HSA_HIP(hipEventRecord(ix->ev_split, st));   // the main pass only
    if (P.wide) launch_search<uint16_t, IT>(P, A, st);
    else launch_search<uint8_t, IT>(P, A, st);
    HSA_HIP(hipGetLastError());
    if (lazy) {
        // the forward pass: the forward rows and the forward-strand searches of the reads
        // the main pass listed (count on the device; queue head ctr[6]); its overflows go
        // to the same re-run list as the main pass's
        SearchArgs F = A;
        F.job_list = A.fwd_list; F.n_dev = d_fwd_n; F.qctr = 6; F.fwd_only = 1;
        F.fwd_list = nullptr; F.fwd_n = nullptr; F.wkey = nullptr; F.perm = nullptr; F.rmap = nullptr;
        const unsigned rblocks = (unsigned)(((size_t)n + BLOCK - 1) / BLOCK);
        if (P.wide) hipLaunchKernelGGL((k_widths_reads<uint16_t, IT>), dim3(rblocks), dim3(BLOCK), 0, st, F, 2u, d_list2, d_n2);
        else hipLaunchKernelGGL((k_widths_reads<uint8_t, IT>), dim3(rblocks), dim3(BLOCK), 0, st, F, 2u, d_list2, d_n2);
        HSA_HIP(hipGetLastError());
        if (P.wide) launch_search<uint16_t, IT>(P, F, st);
        else launch_search<uint8_t, IT>(P, F, st);
        HSA_HIP(hipGetLastError());
    }
    if (split) {
        const unsigned nb = (unsigned)(((size_t)n + BLOCK - 1) / BLOCK);
        hipLaunchKernelGGL(k_split_finalize, dim3(nb), dim3(BLOCK), 0, st, A);
        HSA_HIP(hipGetLastError());
        if (getenv("HSA_VERBOSE")) {
            fprintf(stderr, "[hsa] strand-split main pass: %d reads on %zu lanes\n", n, P.lanes);
            if (A.fr_c) {
                unsigned long long c[9];
                HSA_HIP(hipMemcpyAsync(c, A.fr_c, sizeof c, hipMemcpyDeviceToHost, st));
                HSA_HIP(hipStreamSynchronize(st));
                fprintf(stderr, "[hsa] helpers: %llu offers (%llu refused), %llu chunks, %llu sub-searches, %llu strands "
                                "answered by them, %llu rank queries in sub-searches\n", c[4], c[5], c[0], c[6], c[7], c[8]);
            }
        }
    }
    return 0;
}

static bool any_gaps(const hsa_regime_t *rg, int n)
{
    for (int r = 0; r < n; ++r)
        if (rg[r].max_gapo > 0) return true;
    return false;
}

// 16-bit pruning elements when a bid may be compared with a bound above 14 (WFmt).
static bool need_wide(const hsa_regime_t *rg, int n)
{
    for (int r = 0; r < n; ++r)
        if (rg[r].max_diff > 14 || rg[r].max_seed_diff > 14) return true;
    return false;
}

// 4-bit pruning elements are exact while every bid comparison bound is <= 6 (WFmt<WNib>);
// a job's max_diff never exceeds its regime's
static bool nib_exact(const hsa_regime_t *rg, int n)
{
    for (int r = 0; r < n; ++r)
        if (rg[r].max_diff > 6 || rg[r].max_seed_diff > 6) return false;
    return true;
}

static int jobs_limits(const hsa_job_t *jobs, int n, int &max_len, int &max_seed)
{
    max_len = 0; max_seed = 0;
    for (int j = 0; j < n; ++j) {
        if (jobs[j].len > ANY_MAX_LEN) { hsa_set_error("read %d longer than %d (gap_entry_t.info, bwtgap.c:157)", j, ANY_MAX_LEN); return HSA_E_ARG; }
        if (jobs[j].max_diff < -1) { hsa_set_error("max_diff out of range"); return HSA_E_ARG; }
        if ((int)jobs[j].len > max_len) max_len = (int)jobs[j].len;
        if ((int)jobs[j].len > jobs[j].seed_len && jobs[j].seed_len > max_seed) max_seed = jobs[j].seed_len;
    }
    return 0;
}

// regimes + bucket maps into the staging area: [regimes (256 B)][bmap 2*MAXS].
// Repeated launches with the same options skip the copy (a pageable H2D copy
// would otherwise wait for the stream and stall the host between launches).
static int stage_regimes(hsa_index *ix, const hsa_regime_t *regimes, int n_regimes, char *dst, int &nb,
                         hipStream_t st, bool force)
{
    static_assert(256 + 2 * MAXS <= sizeof(ix->staged), "staging copy");
    uint8_t host[256 + 2 * MAXS];
    memset(host, 0xFF, sizeof host);
    memcpy(host, regimes, sizeof(hsa_regime_t) * n_regimes);
    nb = 1;
    int ntab = 8;
    for (int r = 0; r < n_regimes; ++r) {
        int k = bucket_map(regimes[r], host + 256 + r * MAXS);
        nb = k > nb ? k : nb;
        ntab = regimes[r].n_stacks > ntab ? regimes[r].n_stacks : ntab;
    }
    if (nb > MAXB) { hsa_set_error("%d reachable scores: at most %d stack buckets", nb, MAXB); return HSA_E_ARG; }
    ix->staged_ntab = (ntab + 7) / 8 * 8;
    ix->staged_mmb = mm_buckets(regimes, n_regimes, host + 256);
    ix->staged_min_entries = regimes[0].max_entries;
    for (int r = 1; r < n_regimes; ++r)
        if (regimes[r].max_entries < ix->staged_min_entries) ix->staged_min_entries = regimes[r].max_entries;
    if (!force && ix->staged_valid && memcmp(ix->staged, host, sizeof host) == 0) return 0;
    memcpy(ix->staged, host, sizeof host);
    ix->staged_valid = 1;
    HSA_HIP(hipMemcpyAsync(dst, ix->staged, sizeof host, hipMemcpyHostToDevice, st));
    HSA_HIP(hipStreamSynchronize(st));
    return 0;
}

// ---------------------------------------------------------------- the k_search_any passes
// Device buffers of one search's k_search_any passes (in ix->d_any_aux): the regimes, the
// counters (0 jobs for k_search, 1 jobs for k_search_any, 2 its queue head, 3 jobs it
// hands to its large-capacity pass, 4 that pass's queue head) and the job lists.
struct AnyBufs {
    hsa_regime_t *reg;
    unsigned long long *cnt;
    int32_t *l_fast, *l_any, *l_ovf;
};

static int any_prepare(hsa_index *ix, const hsa_regime_t *regimes, int n_regimes, size_t n, hipStream_t st, AnyBufs &B)
{
    const size_t lb = (n * 4 + 255) / 256 * 256;
    if (ix->d_any_cap > ((size_t)8 << 30)) {       // a past large pass's stacks: give them back
        HSA_HIP(hipStreamSynchronize(st));
        (void)hipFree(ix->d_any);
        ix->d_any = nullptr;
        ix->d_any_cap = 0;
    }
    int rc = hsa_grow(&ix->d_any_aux, &ix->d_any_aux_cap, 512 + 3 * lb);
    if (rc) return rc;
    char *d = (char *)ix->d_any_aux;
    B.reg = (hsa_regime_t *)d;
    B.cnt = (unsigned long long *)(d + 256);
    B.l_fast = (int32_t *)(d + 512);
    B.l_any = (int32_t *)(d + 512 + lb);
    B.l_ovf = (int32_t *)(d + 512 + 2 * lb);
    HSA_HIP(hipMemcpyAsync(B.reg, regimes, sizeof(hsa_regime_t) * n_regimes, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemsetAsync(B.cnt, 0, 64, st));
    HSA_HIP(hipStreamSynchronize(st));
    return 0;
}

// jobs up to fast_max bases go to k_search's list, longer ones to k_search_any's
static __global__ void __launch_bounds__(BLOCK) k_partition(const hsa_job_t *jobs, int n, uint32_t fast_max,
                                                            int32_t *l_fast, int32_t *l_any, unsigned long long *cnt)
{
    const int j = (int)(blockIdx.x * BLOCK + threadIdx.x);
    if (j >= n) return;
    if (jobs[j].len <= fast_max) l_fast[atomicAdd(&cnt[0], 1ull)] = j;
    else l_any[atomicAdd(&cnt[1], 1ull)] = j;
}

// One k_search_any pass.  big: the large-capacity pass (pools up to the reference's
// max_entries bound, 262 144 hits, few lanes) for the jobs the first pass overflowed.
template <typename IT>
static int any_pass(hsa_index *ix, const AnyBufs &B, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *d_jobs,
                    const int32_t *d_list, const unsigned long long *n_dev, int n_host, size_t n_bound, uint32_t max_len,
                    uint32_t max_seed, const uint8_t *d_codes, const MgPass *mg, int32_t *d_n, uint32_t *d_fl,
                    uint64_t *d_ho, uint32_t *d_hits, uint64_t hit_cap, unsigned long long *d_ctr,
                    unsigned long long *qhead, int32_t *ovf_list, unsigned long long *ovf_n, bool big, hipStream_t st)
{
    if (n_bound == 0) return 0;
    if (big && n_dev) {
        // the large pass's lanes hold whole stacks: size it by the reads that overflowed
        // (one stream sync; this path only runs for reads/regimes k_search cannot hold)
        unsigned long long cnt = 0;
        HSA_HIP(hipMemcpyAsync(&cnt, n_dev, sizeof cnt, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipStreamSynchronize(st));
        if (cnt == 0) return 0;
        n_bound = (size_t)cnt;
    }
    AnyArgs A;
    memset(&A, 0, sizeof A);
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.fwd64 = hsa_rank_dir64(ix, 0);
    A.rev64 = hsa_rank_dir64(ix, 1);
    A.T = ix->T; A.T64 = ix->T64;
    memcpy(A.C, ix->C, sizeof A.C);
    memcpy(A.C64, ix->C64, sizeof A.C64);
    A.regimes = B.reg; A.jobs = d_jobs; A.list = d_list; A.n_dev = n_dev; A.n_host = n_host; A.codes = d_codes;
    A.mg = mg ? mg->d_mg : nullptr; A.cw = mg ? mg->d_cw : nullptr;
    A.n_aln = d_n; A.flags = d_fl; A.hit_off = d_ho; A.hits = d_hits; A.hit_cap = hit_cap; A.ctr = d_ctr;
    A.qhead = qhead; A.ovf_list = ovf_list; A.ovf_n = ovf_n;
    uint32_t nst = 1, max_entries = 0;
    for (int r = 0; r < n_regimes; ++r) {
        nst = (uint32_t)regimes[r].n_stacks > nst ? (uint32_t)regimes[r].n_stacks : nst;
        max_entries = (uint32_t)regimes[r].max_entries > max_entries ? (uint32_t)regimes[r].max_entries : max_entries;
    }
    // capacities: live entries never exceed max_entries + 9 (bwtgap.c:150-151)
    const uint64_t want = (uint64_t)max_entries + 16u;
    static const uint32_t pcap1 = getenv("HSA_ANY_PCAP") ? (uint32_t)atoi(getenv("HSA_ANY_PCAP")) : 8192u;   // A/B only
    const uint32_t pcap = big ? (uint32_t)(want < (4ull << 20) ? want : (4ull << 20)) : pcap1;
    const uint32_t hcap = big ? 262144u : 512u;
    const size_t lb = any_layout<IT>(A, max_len, max_seed, nst, pcap, hcap, 10);
    // the large pass holds whole stacks (~75 MB a lane at max_entries 2 000 000) and its
    // reads are the slow ones: as many lanes as half the free HBM allows, up to 64 GB
    size_t budget = (size_t)4 << 30, lanes_max = 16384;
    if (big) {
        size_t fr = 0, tot = 0;
        HSA_HIP(hipMemGetInfo(&fr, &tot));
        budget = fr / 2 < ((size_t)64 << 30) ? fr / 2 : ((size_t)64 << 30);
        lanes_max = 4096;
    }
    size_t lanes = n_bound < lanes_max ? n_bound : lanes_max;
    if (lanes * lb > budget) lanes = budget / lb;
    if (lanes < 1) lanes = 1;
    A.nlanes = (uint32_t)lanes;
    if (lanes * lb + 256 > ix->d_any_cap) HSA_HIP(hipStreamSynchronize(st));   // a pass may still use the old one
    int rc = hsa_grow(&ix->d_any, &ix->d_any_cap, lanes * lb + 256);
    if (rc) return rc;
    A.scratch = (uint8_t *)ix->d_any;
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] k_search_any%s: %zu lanes x %zu B (pool %u, hits %u, %u stacks, reads <= %u bp)\n",
                big ? " (large pass)" : "", lanes, lb, pcap, hcap, nst, max_len);
    hipLaunchKernelGGL(k_search_any<IT>, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, st, A);
    HSA_HIP(hipGetLastError());
    return 0;
}

// hsa_search_device / hsa_search_device64: the main pass over a device-resident batch,
// then the BIG and HUGE capacity re-runs, all queued on one stream without a host sync.
template <typename IT>
static int search_device_impl(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_device_batch_t *b,
                              void *stream)
{
    // regimes: host array; staged into the index's staging area
    if (n_regimes < 1 || n_regimes > 2) { hsa_set_error("1 or 2 regimes"); return HSA_E_ARG; }
    if (sizeof(IT) == 8 && !ix->wide) { hsa_set_error("not a 64-bit index (hsa_index_create_device64)"); return HSA_E_ARG; }
    int rc = check_regimes(regimes, n_regimes);
    if (rc) return rc;
    if (b->max_len < 1 || b->max_len > ANY_MAX_LEN || b->max_seed < 0 || b->max_seed > ANY_MAX_LEN) {
        hsa_set_error("max_len/max_seed out of range");
        return HSA_E_ARG;
    }
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = stream ? (hipStream_t)stream : ix->stream;
    unsigned long long *ctr = (unsigned long long *)b->d_counters;
    hipEvent_t *pe = ix->pev[ix->pev_n % hsa_index::PASS_RING];
    for (int j = 0; j < 3; ++j)
        if (!pe[j]) HSA_HIP(hipEventCreate(&pe[j]));
    // reads longer than k_search holds, or a regime outside its layouts: k_search_any
    // (all jobs for such a regime; the long ones, partitioned on the device, otherwise)
    const bool fast_rg = fast_regimes(regimes, n_regimes);
    const bool any_path = !fast_rg || (uint32_t)b->max_len > FAST_MAX_LEN;
    AnyBufs AB{};
    if (any_path && (rc = any_prepare(ix, regimes, n_regimes, (size_t)b->n_jobs, st, AB))) return rc;
    if (!fast_rg) {
        ++ix->pev_n;
        HSA_HIP(hipEventRecord(pe[0], st));
        HSA_HIP(hipEventRecord(pe[1], st));
        HSA_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(unsigned long long), st));
        if ((rc = any_pass<IT>(ix, AB, regimes, n_regimes, b->d_jobs, nullptr, nullptr, b->n_jobs, (size_t)b->n_jobs,
                               (uint32_t)b->max_len, (uint32_t)b->max_seed, b->d_codes, nullptr, b->d_n_aln, b->d_flags,
                               b->d_hit_off, b->d_hits, b->hit_cap, ctr, AB.cnt + 2, AB.l_ovf, AB.cnt + 3, false, st)) ||
            (rc = any_pass<IT>(ix, AB, regimes, n_regimes, b->d_jobs, AB.l_ovf, AB.cnt + 3, 0, (size_t)b->n_jobs,
                               (uint32_t)b->max_len, (uint32_t)b->max_seed, b->d_codes, nullptr, b->d_n_aln, b->d_flags,
                               b->d_hit_off, b->d_hits, b->hit_cap, ctr, AB.cnt + 4, nullptr, nullptr, true, st)))
            return rc;
        HSA_HIP(hipEventRecord(pe[2], st));
        return 0;
    }
    const int fast_len = (uint32_t)b->max_len > FAST_MAX_LEN ? (int)FAST_MAX_LEN : b->max_len;
    const int fast_seed = b->max_seed > fast_len ? fast_len : b->max_seed;
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, 1536))) return rc;
    int nb = 0;
    if ((rc = stage_regimes(ix, regimes, n_regimes, (char *)ix->d_in, nb, st, before != ix->d_in))) return rc;
    LaunchPlan P, B, H;
    constexpr uint32_t EB = 4u * sizeof(IT);        // pool entry bytes
    const bool gaps = any_gaps(regimes, n_regimes), wide = need_wide(regimes, n_regimes);
    int max_entries = 0;
    for (int r = 0; r < n_regimes; ++r) max_entries = regimes[r].max_entries > max_entries ? regimes[r].max_entries : max_entries;
    const bool nib_ok = nib_exact(regimes, n_regimes);
    if ((rc = plan_launch(ix, b->n_jobs, fast_len, fast_seed, nb, gaps, wide, PASS_MAIN, P, 0, EB, nib_ok)) ||
        (rc = plan_launch(ix, b->n_jobs, fast_len, fast_seed, nb, gaps, wide, PASS_BIG, B, 0, EB, nib_ok)) ||
        (rc = plan_launch(ix, b->n_jobs, fast_len, fast_seed, nb, gaps, wide, PASS_HUGE, H, max_entries, EB)))
        return rc;
    if ((rc = hsa_grow(&ix->d_ovf, &ix->d_ovf_cap, (size_t)b->n_jobs * 4 + 64)) ||
        (rc = hsa_grow(&ix->d_ovf2, &ix->d_ovf2_cap, (size_t)b->n_jobs * 4 + 64)))
        return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)ix->d_in;
    const uint8_t *d_bmap = (const uint8_t *)ix->d_in + 256;
    ++ix->pev_n;
    ix->ev_split = pe[1];
    HSA_HIP(hipEventRecord(pe[0], st));
    const int32_t *fast_list = nullptr;
    const unsigned long long *fast_n = nullptr;
    if (any_path) {                                  // long reads in the batch: split it on the device
        const unsigned g = (unsigned)(((size_t)b->n_jobs + BLOCK - 1) / BLOCK);
        hipLaunchKernelGGL(k_partition, dim3(g ? g : 1), dim3(BLOCK), 0, st, b->d_jobs, b->n_jobs, FAST_MAX_LEN, AB.l_fast,
                           AB.l_any, AB.cnt);
        HSA_HIP(hipGetLastError());
        fast_list = AB.l_fast;
        fast_n = AB.cnt;
    }
    if ((rc = launch_pass<IT>(ix, P, ix->main, d_reg, d_bmap, b->d_jobs, fast_list, b->n_jobs, fast_len, fast_seed,
                              b->d_codes, b->d_n_aln, b->d_flags, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st,
                              (int32_t *)ix->d_ovf, fast_n)))
        return rc;
    // exact re-runs of the reads that overflowed their lane's capacity: BIG for the
    // main pass's (count ctr[8]), HUGE for BIG's (count ctr[12]); the read counts stay
    // on the device, so an empty re-run is a launch whose lanes exit at once
    if ((rc = launch_pass<IT>(ix, B, ix->big, d_reg, d_bmap, b->d_jobs, (const int32_t *)ix->d_ovf, b->n_jobs,
                              fast_len, fast_seed, b->d_codes, b->d_n_aln, b->d_flags, b->d_hit_off, b->d_hits,
                              b->hit_cap, ctr, st, (int32_t *)ix->d_ovf2, ctr + 8, 9, nullptr, 12)) ||
        (rc = launch_pass<IT>(ix, H, ix->huge, d_reg, d_bmap, b->d_jobs, (const int32_t *)ix->d_ovf2, b->n_jobs,
                              fast_len, fast_seed, b->d_codes, b->d_n_aln, b->d_flags, b->d_hit_off, b->d_hits,
                              b->hit_cap, ctr, st, nullptr, ctr + 12, 15)))
        return rc;
    if (any_path &&
        ((rc = any_pass<IT>(ix, AB, regimes, n_regimes, b->d_jobs, AB.l_any, AB.cnt + 1, 0, (size_t)b->n_jobs,
                            (uint32_t)b->max_len, (uint32_t)b->max_seed, b->d_codes, nullptr, b->d_n_aln, b->d_flags,
                            b->d_hit_off, b->d_hits, b->hit_cap, ctr, AB.cnt + 2, AB.l_ovf, AB.cnt + 3, false, st)) ||
         (rc = any_pass<IT>(ix, AB, regimes, n_regimes, b->d_jobs, AB.l_ovf, AB.cnt + 3, 0, (size_t)b->n_jobs,
                            (uint32_t)b->max_len, (uint32_t)b->max_seed, b->d_codes, nullptr, b->d_n_aln, b->d_flags,
                            b->d_hit_off, b->d_hits, b->hit_cap, ctr, AB.cnt + 4, nullptr, nullptr, true, st))))
        return rc;
    HSA_HIP(hipEventRecord(pe[2], st));
    ix->ev_split = ix->evm;
    return 0;
}
