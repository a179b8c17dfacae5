/*
 * hsa_gpu.h -- C ABI of the MI355X search core (libhsa_gpu.so).
 *
 * Plain pointers and sizes only.  This is the layer the reference-compatible
 * entry points (include/hsa_bwtaln.h) are built on, and the layer the Python
 * tests/bench bind with ctypes.
 *
 * What each group replaces in the reference:
 *   hsa_index_*        -- BWTLoad2BWT's in-memory BWT + Occ tables (2BWT-Interface.c:13,
 *                         BWT.c:107): uploaded once to HBM and re-laid out into 16-byte
 *                         rank blocks (3 x u32 counts + 16 two-bit codes).
 *   hsa_occ4_batch     -- BWTAllOccValue (BWT.c:793) for a batch of positions.
 *   hsa_step_batch     -- BWTAllSARangesBackward_Bidirection (2BWT-Interface.c:235).
 *   hsa_width_batch    -- bwt_cal_width type 1 (bwtaln.c:73-98); hsa_width0_batch: type 0.
 *   hsa_search_batch   -- the per-read loop of bwa_cal_sa_reg_gap (bwtaln.c:303-373):
 *                         rc strand then forward strand, bwt_cal_width x2 and
 *                         bwt_match_gap (bwtgap.c:118-331) per strand (two kernels:
 *                         the widths of every read and strand, then the searches).
 *   hsa_match_gap_batch -- bwt_match_gap (bwtgap.c:118-331) called directly with the
 *                         caller's widths, as the splice path calls it (bwtgap.c:812,
 *                         :919, :1192).
 *   hsa_splice_seeds_device -- the six seed searches of bwt_splice_match
 *                         (bwtgap.c:797-812) for every fallback read of a device batch.
 *   hsa_sa_position_*  -- BWTSaValue (BWT.c:1195) + BWTRetrievePositionFromSAIndex
 *                         (2BWT-Interface.c:329).
 *   hsa_extend_batch   -- bwt_extend_backward / bwt_extend_foreward (bwtgap.c:640-663,
 *                         bwt_backtracing_search :346-511): the splice path's seed
 *                         extensions.
 *
 * Errors: every call returns 0 on success or a negative HSA_E* code and leaves a
 * message readable with hsa_last_error().  The library never falls back to a CPU
 * path: without a usable gfx950 device the calls fail.
 */
#ifndef HSA_GPU_H
#define HSA_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HSA_E_HIP     (-1)   /* a HIP runtime call failed */
#define HSA_E_ARG     (-2)   /* invalid argument / unsupported option range */
#define HSA_E_NODEV   (-3)   /* no GPU visible */
#define HSA_E_MEM     (-4)   /* device allocation failed */

/* Search options of one regime (the fields of gap_opt_t the search reads,
 * bwtaln.h:133-143).  max_diff and seed_len are per read (hsa_job_t). */
typedef struct {
    int32_t s_mm, s_gapo, s_gape;
    int32_t mode;                 /* BWA_MODE_* bits: GAPE 0x1, LOGGAP 0x4, NONSTOP 0x10 */
    int32_t indel_end_skip, max_del_occ, max_entries;
    int32_t max_gapo, max_gape;
    int32_t max_seed_diff, max_top2;
    int32_t n_stacks;             /* aln_score(max_diff+1, max_gapo+1, max_gape+1) of the batch's local_opt */
    int32_t max_diff;             /* upper bound of the per-read max_diff of this regime's reads */
} hsa_regime_t;

/* One read to search.  `off` indexes the codes buffer given to hsa_search_batch. */
typedef struct {
    uint64_t off;
    uint32_t len;
    int32_t max_diff;             /* value of aux->opt->max_diff for this read */
    int32_t seed_len;             /* aux->opt->seed_len after bwtaln.c:332 (0x7fffffff = none) */
    int32_t regime;               /* index into the regime array (0 or 1) */
} hsa_job_t;

/* Per-read result flags. */
#define HSA_F_FALLBACK  1u        /* no hit on either strand: caller runs bwt_splice_match */
#define HSA_F_OVERFLOW  2u        /* internal: per-lane stack/hit capacity exceeded (re-run) */

typedef struct hsa_index hsa_index_t;

int         hsa_device_count(void);
const char *hsa_last_error(void);

/* Upload a bidirectional index.  code/rcode are the .bwt payload words (2-bit,
 * MSB-first, ceil(T/16) words; BWT.c:156-181).  C/rC are cumulativeFreq[0..4]. */
int  hsa_index_create(int device, uint32_t T, uint32_t isa0, const uint32_t C[5], const uint32_t *code,
                      uint32_t rT, uint32_t risa0, const uint32_t rC[5], const uint32_t *rcode,
                      hsa_index_t **out);
/* Same, from codes already resident on the device (LSB-first 2-bit, 16 per u32). */
int  hsa_index_create_device(int device, uint32_t T, uint32_t isa0, const uint32_t C[5], const uint32_t *d_code_lsb,
                             uint32_t rT, uint32_t risa0, const uint32_t rC[5], const uint32_t *d_rcode_lsb,
                             hsa_index_t **out);
void hsa_index_free(hsa_index_t *ix);
/* Give back the handle's grown working buffers (search scratch of every capacity pass,
 * the splice prefetch's and splice kernel's buffers) after its stream's work is done;
 * the next call allocates them again.  For a process that hands the GPU's memory to
 * another one between batches (no reference counterpart: the reference has no device).
 * No other call may be in flight on this handle (or use its buffers from another host
 * thread) while it runs: it waits for the stream's queued work only, not for host threads
 * that are about to queue more.  The drop-in entry points never call it. */
int hsa_index_release_scratch(hsa_index_t *ix);
/* The HIP stream (hipStream_t) the library launches on for this index. */
void *hsa_index_stream(const hsa_index_t *ix);
size_t hsa_index_bytes(const hsa_index_t *ix);
int  hsa_index_device(const hsa_index_t *ix);
/* The index's root width trie (hsa_amd/csrc/hsa_trie.h): every string of up to *depth
 * characters with the interval k_widths' forward extension computes for it (0: none;
 * HSA_TRIE_DEPTH at creation, default 12); *sdepth is 0 (k_search takes rank steps
 * only); *bytes of device memory it takes.  Its loads are counted in d_counters[10]. */
int  hsa_index_trie(const hsa_index_t *ix, uint32_t *depth, uint32_t *sdepth, size_t *bytes);
/* A second handle on the same resident index, for passes that run concurrently: the
 * clone shares src's read-only device arrays (rank blocks, wrap tables, trie, SA) and
 * has its own stream, events and search scratch, so hsa_search_device on
 * the two handles may overlap (the next batch's k_widths fills the last waves of this
 * one's k_search).  hsa_index_free(src) while clones are live defers the free of the
 * shared arrays to the last clone's hsa_index_free (src must not be used after it);
 * hsa_index_set_sa refuses a clone and an index with live clones.  No reference
 * counterpart: the reference searches one batch at a time (bwtaln.c:477, :506). */
int  hsa_index_clone(hsa_index_t *src, hsa_index_t **out);

/* Rank/step/width primitives over host arrays (tests and tools). */
int hsa_occ4_batch(hsa_index_t *ix, int dir, size_t n, const uint32_t *pos, uint32_t *occ4_out);
int hsa_step_batch(hsa_index_t *ix, size_t n, const uint32_t *klrr, uint32_t *out16);
int hsa_width_batch(hsa_index_t *ix, size_t n, const uint64_t *offs, const uint32_t *lens,
                    const uint8_t *codes, size_t codes_len, uint32_t *width_out /* 2*(len+1) words per read, packed */);
/* bwt_cal_width type 0 (bwtaln.c:98-115, backward on the forward BWT): entries 1..len
 * as the reference writes them; entry 0, which the reference never writes, is 0. */
int hsa_width0_batch(hsa_index_t *ix, size_t n, const uint64_t *offs, const uint32_t *lens,
                     const uint8_t *codes, size_t codes_len, uint32_t *width_out);

/* One seed extension of the splice path: bwt_extend_backward (dir 1) or
 * bwt_extend_foreward (dir 0), bwtgap.c:640-663 -> bwt_backtracing_search (:346-511).
 * The call extends hit `aln` (bwt_aln1_t words, bwtaln.h:41-50) over `len` read
 * positions toward max_pos (*_left / *_right).  It reads the strand sequence and the
 * direction's width bids (width_back backward, width_fore forward) only inside the
 * read-position window [lo, lo + n) -- backward [min(start - len, max_pos),
 * max(start, max_pos + 1)], forward [min(end, max_pos - 1), max(end + len, max_pos)]
 * (an empty window for a negative len without NONSTOP, whose seed entry stops the
 * search at its first pop) -- given at codes[off .. off + n) and bids[off .. off + n).
 * The regime holds aux->opt's fields with max_diff exact, and n_stacks =
 * aux->stack->n_stacks. */
typedef struct {
    int32_t dir;
    int32_t len;
    int32_t max_pos;
    int32_t regime;
    int32_t lo, n;
    uint64_t off;
    uint32_t aln[9];
    uint32_t pad;
} hsa_ext_job_t;

/* n extensions in one batch (one lane per call; stacks in HBM, grown in capacity
 * passes up to the reference's max_entries bound).  Outputs per call: ret (1, 2 or -1
 * as the reference), max_pos after, and the 9 words of the hit after.  A call whose
 * search the reference leaves undefined (a score past the stack's buckets, a rank
 * position past the text, a read position outside its window) fails the batch with
 * HSA_E_ARG. */
int hsa_extend_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_ext_job_t *jobs, int n,
                     const uint8_t *codes, const int32_t *bids, size_t win_len, int32_t *ret, int32_t *max_pos,
                     uint32_t *aln_out);

/* The same calls in slices: call j works in persistent slot slots[j] (0 <= slot <
 * n_slots; the slots' stacks and states stay on the device between calls with the same
 * n_slots), resumes its saved state when resume[j], and runs at most `budget` pops.
 * ret[j]: 1, 2, -1 (finished: max_pos / aln_out valid), HSA_EXT_CONT (not finished:
 * submit it again with resume set), HSA_EXT_E_CAP (needs more stack than a slot holds:
 * run it through hsa_extend_batch), or another negative code (undefined in the
 * reference).  The job's aln is always the call's original hit.  Every regime's
 * n_stacks must be <= HSA_EXT_SLICE_STACKS (a slot's bucket heads); a caller with a
 * larger regime runs those calls through hsa_extend_batch. */
#define HSA_EXT_CONT  (-999)
#define HSA_EXT_E_CAP (-1001)
#define HSA_EXT_SLICE_STACKS 256
int hsa_extend_sliced(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_ext_job_t *jobs,
                      const int32_t *slots, const uint8_t *resume, int n, const uint8_t *codes, const int32_t *bids,
                      size_t win_len, int n_slots, uint32_t budget, int32_t *ret, int32_t *max_pos, uint32_t *aln_out);

/* Search statistics (summed over the call). */
typedef struct {
    uint64_t rank_queries;        /* Occ evaluations the reference would issue (2 per step) */
    uint64_t blocks_loaded;       /* 64-byte rank blocks actually fetched */
    uint64_t pops;                /* gap_pop calls */
    uint64_t overflow_reruns;     /* reads re-run with large per-read capacity */
    double   kernel_ms;           /* device time of the search kernels (HIP events) */
    double   main_kernel_ms;      /* device time of the main (first) search launch */
    uint64_t main_launches;
} hsa_stats_t;

/* Search `n_jobs` reads.  Host pointers; `codes` holds the 0..255 read codes.
 * Outputs: n_aln[j], flags[j], hit_off[j] (offset in hits, in records) and the
 * packed hits, 9 u32 per record in bwt_aln1_t layout (bwtaln.h:41-50), written to
 * *hits (malloc'd by the library; free with hsa_free).  Returns total hits >= 0. */
long hsa_search_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                      const hsa_job_t *jobs, int n_jobs, const uint8_t *codes, size_t codes_len,
                      int32_t *n_aln, uint32_t *flags, uint64_t *hit_off, uint32_t **hits,
                      hsa_stats_t *stats);

/* Device-resident variant for throughput runs: jobs/codes already on the device,
 * outputs stay on the device (d_hits capacity in records).  Launches on `stream`
 * (a hipStream_t; NULL = the library's stream) and does not synchronise: the
 * caller reads d_counters after the stream completes.
 *
 * d_counters: >= 16 u64 of device scratch, zeroed by the call; the library writes
 *   [1]  hit records allocated (may exceed hit_cap: see [11])
 *   [2]  rank queries the reference algorithm issues for these reads: 2 per
 *        bidirectional step, 2 per width step of every strand it searches
 *        (bwtaln.c:343-359); a read re-run for capacity counts its work twice
 *   [3]  64-byte rank sectors fetched    [4] gap_pop calls
 *   [10] steps answered by a root-trie load instead of rank queries (hsa_index_trie)
 *   [7]  the width queries among [2]
 *   [8]  reads that overflowed their lane's capacity in the main pass (8 192 pool
 *        slots, 32 768 with gap opens), re-run on the device in the BIG pass (65 535
 *        slots, 16 384 hits per read)   [9] the big pass's queue head
 *   [12] reads that overflowed the big pass too, re-run in the HUGE pass: popped
 *        slots reused, so any stack up to max_entries + 16 live entries fits (the
 *        reference's own bound, bwtgap.c:150-151; capped at 4 Mi), 262 144 hits
 *        [15] the huge pass's queue head
 *   [11] reads left UNFINISHED: still over capacity in the huge pass, or their hits
 *        did not fit in d_hits; such a read keeps HSA_F_OVERFLOW, n_aln 0, no hits.
 *        Non-zero means: search those reads again with a larger hit_cap.
 *   [13] width queries of every forward-strand row (computed speculatively)
 *   [14] the part of [13] the reference issues (forward strands searched)
 * Reads past k_search's layouts (longer than 1 023 bases: split off on the device) and
 * regimes past them (n_stacks > 512, > 128 reachable scores, max_gapo > 14, max_diff >
 * 125: every read) run k_search_any (hsa_search_any.h) after k_search, into the same
 * outputs and counters; its large-capacity re-runs count a read's work once.  max_len
 * may be up to 65 535 (gap_entry_t.info's 16-bit position, bwtgap.c:157).
 * d_codes: the read codes; the kernels read whole aligned 16-byte words, so the
 *   buffer must stay readable 16 bytes past the last read's end. */
typedef struct {
    const hsa_job_t *d_jobs; int n_jobs;
    const uint8_t *d_codes;
    int32_t *d_n_aln; uint32_t *d_flags; uint64_t *d_hit_off;
    uint32_t *d_hits; uint64_t hit_cap;
    uint64_t *d_counters;         /* >= 16 u64, see above */
    int32_t max_len, max_seed;    /* longest read, longest seed among the jobs */
} hsa_device_batch_t;
int hsa_search_device(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                      const hsa_device_batch_t *b, void *stream);
/* Device time of the two kernels of the last pass on this index (k_widths, then
 * k_search with its overflow re-run); waits for that pass to finish. */
int hsa_last_pass_ms(hsa_index_t *ix, float *widths_ms, float *search_ms);
/* The same for each of the last n (<= 1024) hsa_search_device passes, oldest first:
 * HIP events recorded on the launch stream around each kernel of every pass. */
int hsa_pass_times(hsa_index_t *ix, int n, float *widths_ms, float *search_ms);
/* Kernel geometry/capacity knobs: 0 leaves a knob unchanged; pool_entries < 0 restores
 * its default (8192 entries per lane, 32768 when gap opens are allowed). */
int hsa_configure(int waves_per_cu, int pool_entries, int hit_cap);

void hsa_free(void *p);

/* Synthetic workload helpers (bench data generation on the device). */
int hsa_synth_genome_device(int device, uint64_t T, uint64_t seed, uint32_t *d_code_lsb);

/* ---- bwt_match_gap with caller-supplied widths (bwtgap.c:118-331) ----
 * The splice path calls bwt_match_gap directly (bwtgap.c:812, :919, :1192) with widths
 * it computed itself -- of the read prefix, not of the searched sequence
 * (bwtgap.c:807) -- with width_seed NULL or aliased to width_back (bwtgap.c:809), and
 * the search mutates width_back through gap_shadow (bwtgap.c:217).  One
 * hsa_mg_job_t per call, next to its hsa_job_t: jobs[j].off/len address the searched
 * sequence itself (aux->seq or aux->rc_seq as aux->strand selects), jobs[j].max_diff
 * and seed_len are the call's opt->max_diff and opt->seed_len. */
#define HSA_SEED_NONE  0          /* width_seed == NULL */
#define HSA_SEED_OWN   1          /* width_seed: its own array, seed_len + 1 entries */
#define HSA_SEED_ALIAS 2          /* width_seed == width_back */
typedef struct {
    uint64_t wb_off;              /* width_back[0..len]: pairs (w, bid) at widths + 2 * wb_off */
    uint64_t ws_off;              /* width_seed[0..seed_len] (HSA_SEED_OWN only) */
    int32_t strand;               /* aux->strand (0 or 1), stamped into the hits (bwtgap.c:235) */
    int32_t seed;                 /* HSA_SEED_* */
} hsa_mg_job_t;

/* One search per job with the caller's widths (bwt_cal_width's bwt_width_t pairs, int32
 * w then bid; bids must be >= 0 as bwt_cal_width produces them).  The jobs' width
 * ranges must not overlap.  widths_out (width_pairs pairs, may equal widths) receives
 * each job's width_back after the search; other entries are left as they are.  Hits
 * as hsa_search_batch, with start = end = 0 (bwt_match_gap leaves them to its caller).
 * Returns the total hit count >= 0. */
long hsa_match_gap_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                         const hsa_mg_job_t *mg, int n_jobs, const uint8_t *codes, size_t codes_len,
                         const int32_t *widths, size_t width_pairs, int32_t *widths_out,
                         int32_t *n_aln, uint64_t *hit_off, uint32_t **hits, hsa_stats_t *stats);

/* ---- the splice path's seed searches on the device ----
 * For every read of a device batch that the main pass flagged HSA_F_FALLBACK, the six
 * seed searches bwt_splice_match can make (bwtgap.c:797-812, restated in
 * hsa_amd/splice.py): seed t of strand s (t = 0, 1, 2; sl = len / 3) searches the
 * strand sequence [t sl, t sl + la) with la = sl (+ len % 3 for t = 2), width_back =
 * width_seed = the widths of the strand's PREFIX of length la, and the seed options
 * (GAPE cleared, no gaps, max_diff = max_seed_diff, seed_len = la) given as one regime.
 * Prefix widths, the calls and their searches all run on the device.  Call 3 s + t of
 * read r is output record 6 r + 3 s + t; records of other reads are left untouched. */
typedef struct {
    const hsa_job_t *d_jobs; int n_jobs;  /* the main pass's reads (off, len) */
    const uint8_t *d_codes;
    const uint32_t *d_flags;              /* the main pass's per-read flags */
    int32_t *d_n_aln; uint64_t *d_hit_off; /* 6 * n_jobs records each */
    uint32_t *d_hits; uint64_t hit_cap;   /* hit records (9 u32) */
    uint64_t *d_counters;                 /* >= 16 u64 of device scratch: [1] hits, [2] rank queries, [4] pops */
    int32_t max_len;                      /* longest read */
} hsa_seed_batch_t;
int hsa_splice_seeds_device(hsa_index_t *ix, const hsa_regime_t *seed_regime, const hsa_seed_batch_t *b, void *stream);

/* ---- the splice path's prefetch of one read batch ----
 * bwt_splice_match (bwtgap.c:748-1332) runs on the host for every read the main search
 * leaves without a hit; before its first seed extension, the searches it can make are
 * determined by the read alone.  This call runs all of them for n such reads in one
 * device pass (replacing, for the host's splice tables, one GPU call per bwt_match_gap /
 * bwt_cal_width / BWTRetrievePositionFromSAIndex the reference makes there):
 *   per read r (codes as bwa_seq_t.seq: 0-3, 4 = N; 3 <= lens[r] <= 3 063) and strand s
 *   (0: the read, 1: its reverse complement, bwtaln.c:326-333),
 *   rows (bwt_width_t pairs, int32 w then bid; row_stride pairs apart, row j of read r
 *     at rows + 2 * (6 r + j) * row_stride):
 *     j = s      bwt_cal_width type 1 of the whole strand (L + 1 pairs, bwtaln.c:84-97);
 *                the width of the strand's prefix of length la is its first la entries
 *                and {0, bid of entry la - 1, + 1};
 *     j = 2 + s  type 1 of the strand's last 12 bases (13 pairs; L >= 12 only);
 *     j = 4 + s  type 0 of the whole strand (L + 1 pairs, entry 0 = 0; bwtaln.c:98-115);
 *   calls (8 per read, call 8 r + c):
 *     c = 3 s + t, t = 0..2: seed t of strand s (bwtgap.c:797-812): the strand's bases
 *       [t sl, t sl + la) (sl = L / 3, la = sl + (t == 2 ? L % 3 : 0)), width_back =
 *       width_seed = the strand prefix's widths of length la, regime seed_rg, max_diff
 *       seed_rg->max_diff, seed_len la;
 *     c = 6 + s: the strand's 12-mer anchor when its seeds' hit pattern is 3 (seeds 0 and
 *       1 hit: its last 12 bases with row 2 + s, bwtgap.c:911-919) or 6 (seeds 1 and 2:
 *       its first 12 with the first 13 entries of row s, :1187-1192), width_seed NULL,
 *       regime anchor_rg, max_diff anchor_max_diff[r];
 *     call_n: hits (bwt_aln1_t records at hits + 9 * call_hit, start = end = 0 as
 *       bwt_match_gap returns them), -1 not searched, -2 not finished (hits past the
 *       buffer, or a stack past the reference's bound): the caller searches it itself;
 *     wafter: the call's width_back after the search (gap_shadow, bwtgap.c:217),
 *       cw_stride pairs per call;
 *   SA (with hsa_index_set_sa): BWTRetrievePositionFromSAIndex of k .. min(l, k + 49) of
 *     every hit of every call, in order (bwt_aln_corelate_check, bwtgap.c:698, :711):
 *     4 u32 each as hsa_sa_position_batch, the call's first at sa + 4 * call_sa.
 * The arrays point into pinned host memory the index owns until its next call. */
typedef struct {
    int n, max_len, row_stride, cw_stride;
    const int32_t *rows;
    const int32_t *call_n;
    const uint64_t *call_hit;
    const uint32_t *hits;
    const int32_t *wafter;
    const uint64_t *call_sa;      /* NULL without an SA */
    const uint32_t *sa;
    uint64_t n_hits, n_sa;
    double kernel_ms;
} hsa_splice_pf_t;
int hsa_splice_prefetch_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg, int n,
                              const uint32_t *lens, const uint64_t *offs, const uint8_t *codes, size_t codes_len,
                              const int32_t *anchor_max_diff, hsa_splice_pf_t *out);

/* ---- the splice path itself on the device ----
 * bwt_splice_match (bwtgap.c:748-1332) for the same n reads: the prefetch pass above,
 * then one persistent kernel that runs each read's seed correlation
 * (bwt_aln_corelate_check, :669), motif scan of the reference (splice_site_search_from_pos,
 * :523), seed extensions (bwt_extend_backward / _foreward, :640-663) and intron-end
 * checks (check_site_by_intron_end, :602) on the device (hsa_amd/csrc/hsa_splice.hip).
 * ext_rg is the extensions' regime: the read's local_opt with max_gape 3 (aux_ext,
 * :776-782; its GAPE bit is the local_opt's, the kernel clears and sets it where the
 * reference does); max_diff per read is anchor_max_diff[r]; n_stacks <=
 * HSA_SP_MAX_STACKS.  Needs hsa_index_set_sa and hsa_index_set_text.
 * res: HSA_SP_RES_WORDS u32 per read: status, n_aln (0, 1 or 2), then res_aln[0] and
 * res_aln[1] (9 words each, bwt_aln1_t) as bwt_splice_match returns them.  status 0: the
 * answer; HSA_SP_* > 0: not answered (the reference's code leaves that read undefined
 * here, or it outgrew the kernel's per-lane stack of HSA_SPLICE_CAP entries, or a
 * prefetched search of it did not finish) -- run the host's bwt_splice_match for it
 * (with hsa_splice_prefetch_batch of those reads for its tables).  `pf` receives the
 * pass's shape and kernel_ms only (no tables). */
#define HSA_SP_RES_WORDS 20
#define HSA_SP_MAX_STACKS 128
#define HSA_SP_OK     0
#define HSA_SP_CALL   1   /* a seed or anchor search of the read did not finish */
#define HSA_SP_CAP    2   /* an extension outgrew the per-lane stack */
#define HSA_SP_SCORE  3   /* an extension entry's score past the stack's buckets */
#define HSA_SP_RANK   4   /* a rank position past the text */
#define HSA_SP_WIN    5   /* a read or width position outside the read */
#define HSA_SP_SA     6   /* an SA position in no chromosome block (stale seq id in the reference) */
#define HSA_SP_TEXT   7   /* a text position past the packed reference */
#define HSA_SP_LOOP   8   /* a loop bound the reference does not keep (u32 wrap, buffer) */
int hsa_index_set_text(hsa_index_t *ix, const uint32_t *packed, uint64_t n_words, uint32_t dna_len);
typedef struct {
    double kernel_ms;             /* the splice kernel's device time */
    uint64_t extensions, pops, sa_lookups, not_answered;
} hsa_splice_stats_t;
/* The same for a device batch: the reads the main pass (hsa_search_device) left with
 * HSA_F_FALLBACK and no hit go through the prefetch pass and the splice kernel, all on
 * the device and without a host round trip.  d_res: HSA_SP_RES_WORDS u32 per job of the
 * batch, written for those reads only; d_counters (>= 8 u64): [0] reads sent to the
 * splice path, [1] extensions, [2] extension pops, [3] SA lookups, [4] reads not answered,
 * [5] rank queries of the seed and anchor searches with their widths, [6] their hits.
 * Each read's max_diff is its job's; max_len the longest read (3 * 1021 at most): a
 * fallback job shorter than 3 or longer than max_len is not taken and gets HSA_SP_WIN. */
typedef struct {
    const hsa_job_t *d_jobs; int n_jobs;
    const uint8_t *d_codes;
    const uint32_t *d_flags;              /* the main pass's per-read flags */
    const int32_t *d_n_aln;               /* the main pass's per-read hit counts */
    uint32_t *d_res;
    uint64_t *d_counters;
    int32_t max_len;
} hsa_splice_batch_t;
int hsa_splice_device(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg,
                      const hsa_regime_t *ext_rg, const hsa_splice_batch_t *b, void *stream);
int hsa_splice_match_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg,
                           const hsa_regime_t *ext_rg, int n, const uint32_t *lens, const uint64_t *offs,
                           const uint8_t *codes, size_t codes_len, const int32_t *anchor_max_diff, hsa_splice_pf_t *pf,
                           uint32_t *res, hsa_splice_stats_t *stats);

/* SA index -> text position (BWTSaValue BWT.c:1195 + BWTRetrievePositionFromSAIndex
 * 2BWT-Interface.c:329), batched.  hsa_index_set_sa uploads the sampled suffix array
 * as BWTLoad holds it (values[0] = -1, (T+s)/s values, interval s) and the chromosome
 * block table (n_blocks rows of u32 chrID, blockStart, blockEnd, ori; ChrBlock
 * HSP.h:41-46).  Output: 4 u32 per index -- SA value, chrID, 1-based position in the
 * chromosome, position in the packed text; chrID and position are 0xFFFFFFFF when no
 * block holds it. */
int hsa_index_set_sa(hsa_index_t *ix, const uint32_t *sa_values, uint64_t n_values, uint32_t interval,
                     const uint32_t *blocks, int n_blocks);
int hsa_sa_position_batch(hsa_index_t *ix, size_t n, const uint32_t *sa_index, uint32_t *out4);
int hsa_sa_position_device(hsa_index_t *ix, size_t n, const uint32_t *d_sa_index, uint32_t *d_out4, void *stream);

/* Roofline probe: measured rate of uniformly random 64-byte-sector gathers over a
 * table of `table_bytes` (the access pattern of rank queries), in GB/s of sectors
 * touched (sectors/s x 64 B), all CUs at 16 waves each.  per_sector = 1: one 16-byte
 * load per sector (what a rank query issues); 2: four adjacent lanes load the four
 * 16-byte quarters of one sector (16 sectors per wave instruction); 4: each lane
 * loads its whole sector in four loads.  The denominator the search kernel's
 * achieved bandwidth is compared with next to the 8 TB/s spec peak (SURVEY.md §8d;
 * DESIGN.md "The random-access ceiling"). */
int hsa_probe_gather(int device, uint64_t table_bytes, int per_sector, double *gbps);

/* ---- 64-bit intervals (texts of 2^32 characters or more; config 5) ----
 * The reference's bwtint_t is 32-bit (2BWT-Interface.h:26), so its index, its hit
 * record and the drop-in ABI (hsa_bwtaln.h) end at 2^32 - 1 characters.  These entry
 * points run the same search with 64-bit SA intervals.
 *
 * hsa_index_create_device64: as hsa_index_create_device, with 64-bit lengths, '$'
 * rows and C tables, T and rT under 2^36 (HSA_E_ARG otherwise).  The rank blocks keep
 * their counts modulo 2^32 and a wrap table (the blocks where a base count passes a
 * multiple of 2^32, found at creation, 512 bytes in front of the blocks) restores the
 * high part.  An index under 2^32 characters also serves every 32-bit entry point; a
 * longer one only the *64 ones (the others return HSA_E_ARG). */
int hsa_index_create_device64(int device, uint64_t T, uint64_t isa0, const uint64_t C[5], const uint32_t *d_code_lsb,
                              uint64_t rT, uint64_t risa0, const uint64_t rC[5], const uint32_t *d_rcode_lsb,
                              hsa_index_t **out);
int hsa_index_is64(const hsa_index_t *ix);
/* BWTAllOccValue (BWT.c:793) at 64-bit positions 0..T+1: 4 u64 per position. */
int hsa_occ4_batch64(hsa_index_t *ix, int dir, size_t n, const uint64_t *pos, uint64_t *occ4_out);
/* The hit record of the 64-bit search: bwt_aln1_t (bwtaln.h:41-50) with 64-bit
 * k, l, rev_k, rev_l; 14 u32 (56 bytes). */
typedef struct {
    uint32_t n_mm:16, n_gapo:8, n_gape:8;
    uint32_t type:30, strand:2;
    uint64_t k, l, rev_k, rev_l;
    int32_t start, end;
    int32_t score, pad;
} hsa_aln64_t;
/* hsa_search_device on a 64-bit index (hsa_index_create_device64): the same batch
 * and counters; d_hits holds hit_cap hsa_aln64_t records. */
int hsa_search_device64(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                        const hsa_device_batch_t *b, void *stream);

/* Suffix-array based BWT construction on the device for a text given as LSB-first
 * 2-bit codes (16 per u32).  Produces the $-less BWT codes (LSB-first) and
 * inverseSa0 = rank of suffix 0 among T+1 suffixes incl. '$' (BWT.h:61-83).
 * `reverse` builds the BWT of the reversed text. */
int hsa_build_bwt_device(int device, uint64_t T, const uint32_t *d_text_lsb, int reverse,
                         uint32_t *d_bwt_lsb, uint32_t *isa0, uint32_t C[5]);
/* The BWT of the text as given (no reversal) and, when d_sa is given, its sampled
 * suffix array as `HSA index` stores it (BWTGenerateSaValue, BWTConstruct.c:1241):
 * d_sa[r / sa_interval] = SA[r] for every row r > 0 with r % sa_interval == 0 (row 0,
 * the '$' row, is the caller's: SA = T).  T < 2^32 - 1 (the .sa values are u32). */
int hsa_build_bwt_index_device(int device, uint64_t T, const uint32_t *d_text_lsb, uint32_t *d_bwt_lsb,
                               uint64_t *isa0, uint64_t C[5], uint32_t sa_interval, uint32_t *d_sa);
/* The same for any T >= 1 (64-bit '$' row and C table); d_bwt_lsb holds ceil(T/16)
 * words.  Device memory besides the text and the output: about T bytes plus 9 GB
 * (u64 suffix positions past 2^32 characters). */
int hsa_build_bwt_device64(int device, uint64_t T, const uint32_t *d_text_lsb, int reverse,
                           uint32_t *d_bwt_lsb, uint64_t *isa0, uint64_t C[5]);

#ifdef __cplusplus
}
#endif
#endif
