// hsa_internal.h -- host-side internals shared by the library's HIP sources.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/hsa_gpu.h"
#include "hsa_device.h"
#include "hsa_sa.h"

void hsa_set_error(const char *fmt, ...);

#define HSA_HIP(call)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            hsa_set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return HSA_E_HIP;                                                               \
        }                                                                                   \
    } while (0)

// Per-launch scratch of the search kernel: grows, never shrinks.
// Sized in entries (lanes x per-lane capacity): a launch indexes lane-interleaved
// slots up to its own lanes * pcap, so a wide seed pass and a deep gapped pass share
// one allocation instead of the product of their maxima.
struct SearchScratch {
    size_t pool_entries = 0, hit_entries = 0;
    uint4 *pool = nullptr;       // pool_entries
    void *nxt = nullptr;         // pool_entries links: uint16_t (main, big passes) or uint32_t (huge pass)
    uint32_t *hbuf = nullptr;    // hit_entries * 9
    size_t link_bytes = 2;
};

struct hsa_index {
    int device = 0;
    uint32_t T = 0, isa0 = 0, C[5] = {0, 0, 0, 0, 0};
    uint32_t rT = 0, risa0 = 0, rC[5] = {0, 0, 0, 0, 0};
    uint4 *blk[2] = {nullptr, nullptr};        // HSA_WRAP_HEAD bytes into blk_base
    void *blk_base[2] = {nullptr, nullptr};
    size_t nblk[2] = {0, 0};
    // 64-bit interval index (hsa_index_create_device64): exact lengths / counts and the
    // wrap tables of RankDir64 (hsa_device.h).  is64: a text of 2^32 characters or
    // more, which only the *64 entry points accept.
    bool wide = false, is64 = false;
    uint64_t T64 = 0, isa0_64 = 0, C64[5] = {0, 0, 0, 0, 0};
    uint64_t rT64 = 0, risa0_64 = 0, rC64[5] = {0, 0, 0, 0, 0};
    bool any_wrap[2] = {false, false};         // a wrap table entry (RankDir64)
    hipStream_t stream = nullptr;
    int n_cu = 0;
    SearchScratch main, big, huge;
    void *d_ovf2 = nullptr; size_t d_ovf2_cap = 0; // device path: reads the big pass hands to the huge pass
    // staging for the host-pointer batch API
    void *d_in = nullptr; size_t d_in_cap = 0;
    void *d_out = nullptr; size_t d_out_cap = 0;
    // per-(read, strand) width rows written by k_widths, read by k_search
    void *d_wrows = nullptr; size_t d_wrows_cap = 0;
    void *d_ovf = nullptr; size_t d_ovf_cap = 0;   // device-path list of reads to re-run
    void *d_seed = nullptr; size_t d_seed_cap = 0; // splice seed calls (hsa_splice_seeds_device)
    void *d_ext = nullptr; size_t d_ext_cap = 0;   // seed-extension stacks (hsa_extend_batch)
    void *d_slices = nullptr; size_t d_slices_cap = 0; // persistent extension slots (hsa_extend_sliced)
    // k_search_any (hsa_search_any.h): per-lane scratch, job lists and counters, regimes
    void *d_any = nullptr; size_t d_any_cap = 0;
    void *d_any_aux = nullptr; size_t d_any_aux_cap = 0;
    void *d_split = nullptr; size_t d_split_cap = 0;   // strand-split items' results (k_split_finalize)
    void *d_help = nullptr; size_t d_help_cap = 0;     // strand-split tails: the shared frontier (k_search helpers)
    void *d_fwd = nullptr; size_t d_fwd_cap = 0;       // lazy forward rows: count + reads for the forward pass
    // hsa_splice_prefetch_batch: inputs, calls and outputs; its SA lookups; the pinned
    // host copy of the outputs the caller's tables point into
    void *d_pf = nullptr; size_t d_pf_cap = 0;
    void *d_pf2 = nullptr; size_t d_pf2_cap = 0;
    void *h_pf = nullptr; size_t h_pf_cap = 0;
    // sampled suffix array + chromosome blocks (SA -> position, hsa_sa.hip)
    uint32_t *d_sa = nullptr, *d_blocks = nullptr;
    uint32_t sa_interval = 0, n_blocks = 0;
    // the packed text as the host's HSP holds it (hsa_index_set_text): 16 codes per u32,
    // the first in the high bits, text_words words as allocated (DNALoadPacked,
    // TextConverter.c:704-707), dna_len the HSP's dnaLength
    uint32_t *d_text = nullptr;
    uint64_t text_words = 0;
    uint32_t dna_len = 0;
    // the splice path's kernel (hsa_splice.hip): per-lane state, stacks, buffers
    void *d_sp = nullptr; size_t d_sp_cap = 0;
    uint64_t *d_ctr = nullptr;
    // the root width trie (hsa_trie.h): every string of up to trie_depth characters;
    // built with the index's interval width (trie_wide: 64-bit entries), 0 = none
    void *d_trie_w = nullptr;           // entries of levels 1..D
    uint32_t trie_depth = 0;
    bool trie_wide = false;
    size_t trie_bytes = 0;
    unsigned char staged[1280];         // last regime block copied to d_in (skip identical re-copies)
    int staged_valid = 0;
    bool staged_mmb = false;            // staged regimes: bucket == n_mm (see mm_buckets)
    int staged_ntab = 128;              // staged regimes: score table entries per regime (k_search LDS)
    int staged_min_entries = 0;         // staged regimes: the smallest max_entries (helpers need > the pool)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t evm = nullptr;           // between k_widths and k_search of the last pass (timing split)
    hipEvent_t ev_sp = nullptr;         // after the splice kernel (hsa_splice_match_batch: ev1 .. ev_sp)
    // hsa_search_device passes: start / between k_widths and k_search / end, per pass, in a
    // ring (hsa_pass_times), so a caller can time every launch of a back-to-back run
    static constexpr int PASS_RING = 1024;
    hipEvent_t pev[PASS_RING][3] = {};
    uint64_t pev_n = 0;
    hipEvent_t ev_split = nullptr;      // recorded by launch_pass between k_widths and k_search
    // hsa_index_clone: a clone shares the parent's read-only device arrays (rank blocks
    // and wrap tables, tries, SA) and owns its stream, events and scratch
    hsa_index *parent = nullptr;
    int n_clones = 0;                   // live clones of this index
    bool free_pending = false;          // hsa_index_free called while clones were live
};
// HSA_E_ARG when an index's shared arrays may not be replaced (a clone, or an index with
// live clones)
int hsa_need_unshared(const hsa_index *ix, const char *what);

int hsa_grow(void **p, size_t *cap, size_t need);
int hsa_realloc_device(void **out, void **old, size_t bytes);
// hsa_mg_job_t.ws_off of an HSA_SEED_ALIAS job whose width_back is the first len entries
// of a longer row (internal: the splice seeds, hsa_search.hip): terminal computed, no export
#define HSA_MG_PREFIX 0xFFFFFFFFFFFFFFFFull
SaView hsa_sa_view(const hsa_index *ix);

// The splice prefetch's device outputs (hsa_splice_prefetch_batch, hsa_search.hip), as
// the splice path's kernel reads them (hsa_splice.hip).
struct PfDev {
    uint32_t n, max_len, sc, rs, cws;
    const uint32_t *lens;
    const int32_t *amd;            // per read: its local_opt max_diff
    const uint8_t *scodes;         // strand s of read r at (2 r + s) sc
    const int32_t *rows;           // 6 rows per read, rs pairs each
    const int32_t *cw;             // per call: width_back after gap_shadow, cws pairs
    const int32_t *call_n;         // 8 calls per read: seeds 0-5, anchors 6-7 (-1: not searched)
    const uint32_t *call_fl;
    const uint64_t *call_hit;      // record index in hits_s (seeds) / hits_a (anchors)
    const uint32_t *hits_s, *hits_a;
    const unsigned long long *d_n; // the reads' count on the device (hsa_splice_device), or null: n
    const int32_t *idx;            // answer of read r at res[idx[r]] (hsa_splice_device), or null: r
};
// bwt_splice_match for the prefetch's reads on the device (d_res: HSA_SP_RES_WORDS u32
// per read); ext_rg: the extension regime (local_opt with max_gape 3, bwtgap.c:777-782)
int hsa_splice_device_launch(hsa_index *ix, const PfDev &pd, const hsa_regime_t &ext_rg, uint32_t *d_res,
                             unsigned long long *d_ctr, hipStream_t st);
int hsa_scratch_reserve(SearchScratch &s, size_t lanes, size_t pcap, size_t hcap, size_t link_bytes = 2);
void hsa_scratch_free(SearchScratch &s);
// HSA_E_ARG unless the index fits the 32-bit entry points (bwtint_t, 2BWT-Interface.h:26)
int hsa_need32(const hsa_index *ix);
RankDir64 hsa_rank_dir64(const hsa_index *ix, int dir);   // the wrap-table rank of a wide index

// Knobs (hsa_configure).
extern int g_waves_per_cu;
extern int g_pool_entries;
extern int g_batch_k;
extern int g_batch_idle;
extern int g_hit_cap;
