/*
 * hsa_oracle.c -- plain-C restatement of the HSA inexact-alignment path.
 *
 * TEST INFRASTRUCTURE ONLY (see hsa_oracle.h).  Each function cites the
 * reference file:line it restates.  It favours obviousness over speed: the rank
 * structure is a flat prefix count every 32 characters, the stack is the
 * reference's bucketed LIFO with realloc'd buckets.
 *
 * Parity pin: tests/test_oracle.py checks every function here against the
 * golden vectors the compiled reference produced (tests/golden/).
 *
 * Compiled twice: liboracle.so (or_*: 32-bit intervals, the reference's bwtint_t,
 * 2BWT-Interface.h:26) and, with -DOR_WIDE, liboracle64.so (or64_*: the same
 * algorithm with 64-bit intervals, for texts of 2^32 characters or more, which the
 * reference cannot index -- config 5).  The 64-bit build is pinned against the
 * 32-bit one on the same sub-2^32 indexes (tests/test_oracle.py).
 */
#include "hsa_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef OR_WIDE
typedef uint64_t bw_t;     /* SA interval bound */
typedef int64_t cnt_t;     /* best_cnt (int in bwtgap.c:127) */
#define OR(name) or64_##name
#define HW 14              /* hsa_aln64_t words */
#define H_START 10
#define H_END 11
#else
typedef uint32_t bw_t;
typedef int cnt_t;
#define OR(name) or_##name
#define HW 9               /* bwt_aln1_t words (bwtaln.h:41-50) */
#define H_START 6
#define H_END 7
#endif

#define MODE_GAPE 0x01
#define MODE_LOGGAP 0x04
#define MODE_NONSTOP 0x10
#define ST_M 0
#define ST_I 1
#define ST_D 2

typedef struct {
    bw_t T, isa0, C[5];
    uint64_t *w;    /* $-less BWT, 32 codes per word, code j at bits 2j..2j+1 */
    bw_t *cnt;      /* cnt[b*4+c] = #c in codes [0, 32b) */
} or_bwt_t;

/* rank queries issued by this thread (statistics only; thread-local so that threads
 * sharing one index do not contend on a counter) */
static __thread uint64_t tl_queries;

#ifdef OR_DEPTH_HIST
/* Experiment build only (liboracle_hist.so, tools/exp/depth_hist.py): rank steps by the
 * length of the string they extend to (the trie depth), and how many of them touch two
 * different 16-character rank blocks.  [0]/[1] search steps (expansions and exact
 * tails), [2]/[3] bwt_cal_width steps (depth since the last reset). */
static __thread uint64_t tl_hist[4][64];
static __thread int tl_depth;
#define HIST_DEPTH(d) (tl_depth = (d) < 63 ? (d) : 63)
static void hist_pair(int which, bw_t i0, bw_t i1, bw_t isa0)
{
    i0 -= (i0 > isa0); i1 -= (i1 > isa0);
    tl_hist[which][tl_depth]++;
    if (i0 / 16 != i1 / 16) tl_hist[which + 1][tl_depth]++;
}
void OR(depth_hist)(uint64_t *out, int reset)
{
    memcpy(out, tl_hist, sizeof tl_hist);
    if (reset) memset(tl_hist, 0, sizeof tl_hist);
}
#else
#define HIST_DEPTH(d) ((void)0)
#define hist_pair(w, a, b, c) ((void)0)
#endif

#ifdef OR_DUP_STATS
/* Experiment build only (liboracle_dup.so, tools/dup_stats.py): how many expansions of a
 * bwt_match_gap search repeat one already made in the same search -- the same node
 * (i, k, l, rk, state) with the same counts (exact), or with counts >= an earlier one's
 * (dominated) -- split by whether the search ends with hits.  [0] expansions, [1] exact
 * repeats, [2] dominated ones, of searches with hits; [3]-[5] of searches without. */
static __thread uint64_t tl_dup[6];
void OR(dup_stats)(uint64_t *out, int reset)
{
    memcpy(out, tl_dup, sizeof tl_dup);
    if (reset) memset(tl_dup, 0, sizeof tl_dup);
}
#endif

struct or_index {
    or_bwt_t f, r;
    int unused;
};

static uint32_t rev_pairs32(uint32_t x)   /* reverse the order of the 16 2-bit fields */
{
    x = (x >> 16) | (x << 16);
    x = ((x & 0xFF00FF00u) >> 8) | ((x & 0x00FF00FFu) << 8);
    x = ((x & 0xF0F0F0F0u) >> 4) | ((x & 0x0F0F0F0Fu) << 4);
    return ((x & 0xCCCCCCCCu) >> 2) | ((x & 0x33333333u) << 2);
}

/* code: .bwt words, char j of a word at bits 31-2j..30-2j (BWT.c:156-181,
 * BWTConstruct.c:1209); or, lsb != 0, LSB-first words (char j at bits 2j..2j+1, the
 * device builder's output). */
static void bwt_init(or_bwt_t *b, bw_t T, bw_t isa0, const bw_t C[5], const uint32_t *code, int lsb)
{
    uint64_t nw = ((uint64_t)T + 31) / 32, ncw = ((uint64_t)T + 15) / 16;
    b->T = T; b->isa0 = isa0;
    memcpy(b->C, C, 5 * sizeof(bw_t));
    b->w = (uint64_t *)calloc(nw + 1, sizeof(uint64_t));
    b->cnt = (bw_t *)calloc((nw + 2) * 4, sizeof(bw_t));
    for (uint64_t q = 0; q < nw; ++q) {
        uint64_t lo = lsb ? code[2 * q] : rev_pairs32(code[2 * q]);
        uint64_t hi = 2 * q + 1 < ncw ? (lsb ? code[2 * q + 1] : rev_pairs32(code[2 * q + 1])) : 0;
        b->w[q] = lo | hi << 32;
    }
    if (T & 31) b->w[nw - 1] &= (1ull << (2 * (T & 31))) - 1;   /* BWTClearTrailingBwtCode */
    bw_t acc[4] = {0, 0, 0, 0};
    for (uint64_t q = 0; q <= nw; ++q) {
        memcpy(b->cnt + q * 4, acc, sizeof acc);
        if (q == nw) break;
        uint64_t x = b->w[q], lo = x & 0x5555555555555555ull, hi = (x >> 1) & 0x5555555555555555ull;
        uint32_t n3 = (uint32_t)__builtin_popcountll(lo & hi);
        uint32_t n1 = (uint32_t)__builtin_popcountll(lo) - n3, n2 = (uint32_t)__builtin_popcountll(hi) - n3;
        uint32_t valid = (q + 1) * 32 <= (uint64_t)T ? 32u : (uint32_t)(T - q * 32);
        acc[0] += valid - n1 - n2 - n3; acc[1] += n1; acc[2] += n2; acc[3] += n3;
    }
}

#ifdef OR_WIDE
or_index_t *or64_index_create(uint64_t T, uint64_t isa0, const uint64_t C[5], const uint32_t *code_lsb,
                              uint64_t rT, uint64_t risa0, const uint64_t rC[5], const uint32_t *rcode_lsb)
{
    or_index_t *ix = (or_index_t *)calloc(1, sizeof(or_index_t));
    bwt_init(&ix->f, T, isa0, C, code_lsb, 1);
    bwt_init(&ix->r, rT, risa0, rC, rcode_lsb, 1);
    return ix;
}
#else
or_index_t *or_index_create(uint32_t T, uint32_t isa0, const uint32_t C[5], const uint32_t *code,
                            uint32_t rT, uint32_t risa0, const uint32_t rC[5], const uint32_t *rcode)
{
    or_index_t *ix = (or_index_t *)calloc(1, sizeof(or_index_t));
    bwt_init(&ix->f, T, isa0, C, code, 0);
    bwt_init(&ix->r, rT, risa0, rC, rcode, 0);
    return ix;
}
#endif

void OR(index_free)(or_index_t *ix)
{
    if (!ix) return;
    free(ix->f.w); free(ix->f.cnt); free(ix->r.w); free(ix->r.cnt); free(ix);
}

void OR(free)(void *p) { free(p); }

/* BWTAllOccValue (BWT.c:793-837): $ is not encoded, so an index past inverseSa0
 * is shifted down by one (BWT.c:690); the sampled-Occ + SSE decode then equals the
 * prefix count #{p < i' : code[p] == c} (checked at every i in [0, T+1] on the
 * fixtures).  Here: prefix count at the 32-char word + popcount inside it. */
static void occ4(const or_bwt_t *b, bw_t i, bw_t o[4])
{
    i -= (i > b->isa0);
    uint64_t q = i >> 5;
    uint32_t r = (uint32_t)(i & 31);
    for (int c = 0; c < 4; ++c) o[c] = b->cnt[q * 4 + c];
    if (r) {
        uint64_t x = b->w[q] & ((1ull << (2 * r)) - 1);
        uint64_t lo = x & 0x5555555555555555ull, hi = (x >> 1) & 0x5555555555555555ull;
        uint32_t n3 = (uint32_t)__builtin_popcountll(lo & hi);
        uint32_t n2 = (uint32_t)__builtin_popcountll(hi & ~lo);
        uint32_t n1 = (uint32_t)__builtin_popcountll(lo & ~hi);
        o[0] += r - n1 - n2 - n3; o[1] += n1; o[2] += n2; o[3] += n3;
    }
}

void OR(occ4)(const or_index_t *ix, int dir, bw_t i, bw_t occ[4])
{
    occ4(dir ? &ix->r : &ix->f, i, occ);
}

#ifndef OR_WIDE   /* SA -> position: the 32-bit path only (hsa_sa.hip) */
/* BWTPsiMinusValue (BWT.c:1142-1162) via BWTOccValueOnSpot (BWT.c:924-959): for
 * index != inverseSa0, i = index + 1 shifted past '$' (BWT.c:949), c = the BWT
 * character before i, result C[c] + Occ(c, i) (the count includes that character). */
static uint32_t psi_minus(const or_bwt_t *b, uint32_t index)
{
    if (index == b->isa0) return 0;
    uint32_t i = index + 1;
    i -= (i > b->isa0);
    uint32_t p = i - 1, c = (uint32_t)((b->w[p >> 5] >> (2 * (p & 31))) & 3u);
    /* Occ over the $-less prefix [0, i): occ4 takes a $-including index, so pass the
     * index that shifts back to i */
    uint32_t o[4];
    occ4(b, i + (i > b->isa0 ? 1u : 0u), o);
    return b->C[c] + o[c];
}

/* BWTSaValue (BWT.c:1195-1220): LF-walk to a sampled SA index, then add the steps.
 * sa_values[0] is -1 (BWT.c:222) and PsiMinus(inverseSa0) = 0, so the walk through
 * '$' lands on that sample with u32 wrap-around, exactly as the reference. */
uint32_t or_sa_value(const or_index_t *ix, const uint32_t *sa_values, uint32_t interval, uint32_t sa_index)
{
    uint32_t skipped = 0;
    while (sa_index % interval != 0) {
        ++skipped;
        sa_index = psi_minus(&ix->f, sa_index);
    }
    return sa_values[sa_index / interval] + skipped;
}

/* BWTRetrievePositionFromSAIndex (2BWT-Interface.c:329-361): SA value, then the
 * reference's binary search over the chromosome blocks (rows chrID, blockStart,
 * blockEnd, ori; h starts at nblock).  seq_id / ori_pos are written only when a block
 * holds the position.  Where the reference would read blockList[nblock] (past its
 * end: undefined), the restatement stops as "not found". */
void or_sa_position(const or_index_t *ix, const uint32_t *sa_values, uint32_t interval, const uint32_t *blocks,
                    int n_blocks, uint32_t sa_index, uint32_t *seq_id, uint32_t *ori_pos, uint32_t *occ_pos)
{
    uint32_t occ = or_sa_value(ix, sa_values, interval, sa_index);
    uint32_t l = 0, h = (uint32_t)n_blocks, m, start, end;
    *occ_pos = occ;
    while (l <= h) {
        m = (h + l) >> 1;
        if (m >= (uint32_t)n_blocks) break;
        if ((start = blocks[4 * m + 1]) > occ) {
            h = m - 1;
        } else if ((end = blocks[4 * m + 2]) < occ) {
            l = m + 1;
        } else if (start <= occ && end >= occ) {
            *seq_id = blocks[4 * m];
            *ori_pos = occ - start + blocks[4 * m + 3] + 1;
            break;
        } else {
            break;
        }
    }
}
#endif

/* BWTAllSARangesBackward_Bidirection (2BWT-Interface.c:235-272). */
static void step_all(or_index_t *ix, bw_t k, bw_t l, bw_t rk, bw_t rl, bw_t ok[4], bw_t ol[4], bw_t ork[4], bw_t orl[4])
{
    bw_t oL[4], oR[4], oC[4];
    (void)rk;
    occ4(&ix->f, k, oL);
    occ4(&ix->f, l + 1, oR);
    tl_queries += 2;
    hist_pair(0, k, l + 1, ix->f.isa0);
    oC[3] = 0;
    for (int c = 2; c >= 0; --c) oC[c] = oC[c + 1] + oR[c + 1] - oL[c + 1];
    for (int c = 0; c < 4; ++c) {
        ok[c] = ix->f.C[c] + oL[c] + 1;
        ol[c] = ix->f.C[c] + oR[c];
        orl[c] = rl - oC[c];
        ork[c] = orl[c] - (ol[c] - ok[c]);
    }
}

void OR(step_all)(const or_index_t *ix, bw_t k, bw_t l, bw_t rk, bw_t rl, bw_t ok[4], bw_t ol[4], bw_t ork[4],
                   bw_t orl[4])
{
    step_all((or_index_t *)ix, k, l, rk, rl, ok, ol, ork, orl);
}

/* BWTSARangeBackward_Bidirection (2BWT-Interface.c:135-170): one character. */
static void step1(or_index_t *ix, uint32_t c, bw_t *k, bw_t *l, bw_t *rk, bw_t *rl)
{
    bw_t ok[4], ol[4], ork[4], orl[4];
    step_all(ix, *k, *l, *rk, *rl, ok, ol, ork, orl);
    *k = ok[c]; *l = ol[c]; *rk = ork[c]; *rl = orl[c];
}

/* bwt_match_exact (2BWT-Interface.c:365-388), including the write-back guard
 * (:383-386): an output is only written if its incoming value is non-zero (Q1). */
static int match_exact(or_index_t *ix, const uint8_t *seq, int len, bw_t *sk, bw_t *sl, bw_t *srk, bw_t *srl)
{
    bw_t k = *sk, l = *sl, rk = *srk, rl = *srl;
    for (int i = len - 1; i >= 0; i--) {
        if (seq[i] > 3) return 0;
#ifdef OR_DEPTH_HIST
        HIST_DEPTH(tl_depth + 1);
#endif
        step1(ix, seq[i], &k, &l, &rk, &rl);
        if (k > l) break;
    }
    if (k > l) return 0;
    if (*sk) *sk = k;
    if (*sl) *sl = l;
    if (*srk) *srk = rk;
    if (*srl) *srl = rl;
    return (int)(l - k + 1);
}

/* bwt_cal_width, type 1 (bwtaln.c:73-98): forward extension on the REVERSE BWT
 * with the FORWARD C[] (BWTSARangeForeward, 2BWT-Interface.c:121-132). */
static int cal_width(or_index_t *ix, int len, const uint8_t *str, bw_t *w)
{
    bw_t k = 0, l = ix->f.T;
    int bid = 0;
#ifdef OR_DEPTH_HIST
    int j0 = 0;
#endif
    for (int i = 0; i < len; ++i) {
        uint8_t c = str[i];
        if (c < 4) {
            bw_t a[4], b[4];
            occ4(&ix->r, k, a);
            occ4(&ix->r, l + 1, b);
            tl_queries += 2;
#ifdef OR_DEPTH_HIST
            HIST_DEPTH(i - j0 + 1);
            hist_pair(2, k, l + 1, ix->r.isa0);
#endif
            k = ix->f.C[c] + a[c] + 1;
            l = ix->f.C[c] + b[c];
        }
        if (k > l || c > 3) {
            k = 0; l = ix->f.T; ++bid;
#ifdef OR_DEPTH_HIST
            j0 = i + 1;
#endif
        }
        w[2 * i] = l - k + 1;
        w[2 * i + 1] = (bw_t)bid;
    }
    w[2 * len] = 0;
    w[2 * len + 1] = (bw_t)++bid;
    return bid;
}

int OR(cal_width)(const or_index_t *ix, int len, const uint8_t *str, bw_t *width)
{
    return cal_width((or_index_t *)ix, len, str, width);
}

/* bwt_cal_width, type 0 (bwtaln.c:98-115): backward extension on the FORWARD BWT
 * (BWTSARangeBackward, 2BWT-Interface.c:107-118) from the end of str; entry 0 is never
 * written (the loop stops at i > 0). */
int OR(cal_width0)(const or_index_t *cix, int len, const uint8_t *str, bw_t *w)
{
    const or_index_t *ix = cix;
    bw_t k = 0, l = ix->f.T;
    int bid = 0;
    for (int i = len - 1; i > 0; --i) {
        uint8_t c = str[i];
        if (c < 4) {
            bw_t a[4], b[4];
            occ4(&ix->f, k, a);
            occ4(&ix->f, l + 1, b);
            tl_queries += 2;
            k = ix->f.C[c] + a[c] + 1;
            l = ix->f.C[c] + b[c];
        }
        if (k > l || c > 3) { k = 0; l = ix->f.T; ++bid; }
        w[2 * i] = l - k + 1;
        w[2 * i + 1] = (bw_t)bid;
    }
    w[2 * len] = 0;
    w[2 * len + 1] = (bw_t)++bid;
    return bid;
}

void OR(init_opt)(or_opt_t *o)
{
    memset(o, 0, sizeof *o);
    o->s_mm = 3; o->s_gapo = 11; o->s_gape = 4;
    o->max_diff = -1; o->max_gapo = 1; o->max_gape = 6;
    o->indel_end_skip = 5; o->max_del_occ = 10; o->max_entries = 2000000;
    o->mode = 0x01 | 0x02;
    o->seed_len = 32; o->max_seed_diff = 2;
    o->fnr = 0.04f; o->n_threads = 1; o->max_top2 = 30; o->trim_qual = 0;
}

int OR(cal_maxdiff)(int l, double err, double thres)
{
    double elambda = exp(-l * err);
    double sum, y = 1.0;
    int k, x = 1;
    for (k = 1, sum = elambda; k < 1000; ++k) {
        y *= l * err;
        x *= k;
        sum += elambda * y / x;
        if (1.0 - sum < thres) return k;
    }
    return 2;
}

/* ---- bucketed LIFO (bwtgap.c:13-92) ---- */
typedef struct {
    uint32_t info;          /* score<<21 | i */
    uint8_t n_mm, n_gapo, n_gape, state;
    bw_t k, l, rk, rl;
    int last_diff_pos;
} ent_t;
typedef struct { int n, m; ent_t *a; } bucket_t;
typedef struct { int n_stacks, best, n_entries; bucket_t *b; } stack_t_;

#define SCORE(o, m, g, e) ((m) * (o)->s_mm + (g) * (o)->s_gapo + (e) * (o)->s_gape)

static stack_t_ *stack_new(int n_stacks)
{
    stack_t_ *s = (stack_t_ *)calloc(1, sizeof *s);
    s->n_stacks = n_stacks;
    s->b = (bucket_t *)calloc(n_stacks, sizeof(bucket_t));
    for (int i = 0; i < n_stacks; ++i) { s->b[i].m = 4; s->b[i].a = (ent_t *)calloc(4, sizeof(ent_t)); }
    return s;
}

static void stack_del(stack_t_ *s)
{
    for (int i = 0; i < s->n_stacks; ++i) free(s->b[i].a);
    free(s->b); free(s);
}

static void stack_reset(stack_t_ *s)
{
    for (int i = 0; i < s->n_stacks; ++i) s->b[i].n = 0;
    s->best = s->n_stacks; s->n_entries = 0;
}

static void push(stack_t_ *s, int i, bw_t k, bw_t l, bw_t rk, bw_t rl,
                 int n_mm, int n_gapo, int n_gape, int state, int is_diff, const or_opt_t *o)
{
    int score = SCORE(o, n_mm, n_gapo, n_gape);
    if (score < 0 || score >= s->n_stacks) {
        fprintf(stderr, "oracle: push score %d outside %d buckets (undefined in the reference)\n", score, s->n_stacks);
        abort();
    }
    bucket_t *q = s->b + score;
    if (q->n == q->m) { q->m <<= 1; q->a = (ent_t *)realloc(q->a, sizeof(ent_t) * q->m); }
    ent_t *p = q->a + q->n;
    p->info = (uint32_t)score << 21 | (uint32_t)i;
    p->k = k; p->l = l; p->rk = rk; p->rl = rl;
    p->n_mm = (uint8_t)n_mm; p->n_gapo = (uint8_t)n_gapo; p->n_gape = (uint8_t)n_gape;
    p->state = (uint8_t)state;
    p->last_diff_pos = is_diff ? i : 0;
    ++q->n; ++s->n_entries;
    if (s->best > score) s->best = score;
}

static void pop(stack_t_ *s, ent_t *e)
{
    bucket_t *q = s->b + s->best;
    *e = q->a[q->n - 1];
    --q->n; --s->n_entries;
    if (q->n == 0 && s->n_entries) {
        int i;
        for (i = s->best + 1; i < s->n_stacks; ++i) if (s->b[i].n) break;
        s->best = i;
    } else if (s->n_entries == 0) s->best = s->n_stacks;
}

/* gap_shadow (bwtgap.c:94-105) */
static void shadow(bw_t x, bw_t max, int last_diff_pos, bw_t *w)
{
    int j = 0;
    for (int i = 0; i < last_diff_pos; ++i) {
        if (w[2 * i] > x) w[2 * i] -= x;
        else if (w[2 * i] == x) { w[2 * i + 1] = 1; w[2 * i] = max - (bw_t)(++j); }
    }
}

static int int_log2(uint32_t v)   /* bwtgap.c:107-116 */
{
    int c = 0;
    if (v & 0xffff0000u) { v >>= 16; c |= 16; }
    if (v & 0xff00) { v >>= 8; c |= 8; }
    if (v & 0xf0) { v >>= 4; c |= 4; }
    if (v & 0xc) { v >>= 2; c |= 2; }
    if (v & 0x2) c |= 1;
    return c;
}

typedef struct { int n, m; uint32_t *a; } hitv_t;   /* HW words per hit */

/* one hit record: bwt_aln1_t (bwtaln.h:41-50), or hsa_aln64_t (include/hsa_gpu.h) */
static void put_hit(uint32_t *p, const ent_t *e, bw_t k, bw_t l, bw_t rk, bw_t rl, int strand, int score)
{
    memset(p, 0, HW * sizeof(uint32_t));
    p[0] = (uint32_t)e->n_mm | (uint32_t)e->n_gapo << 16 | (uint32_t)e->n_gape << 24;
#ifdef OR_WIDE
    const bw_t v[4] = {k, l, rk, rl};
    p[1] = (uint32_t)(strand & 3) << 30;            /* type 0 */
    for (int j = 0; j < 4; ++j) { p[2 + 2 * j] = (uint32_t)v[j]; p[3 + 2 * j] = (uint32_t)(v[j] >> 32); }
    p[12] = (uint32_t)score;
#else
    p[1] = k; p[2] = l; p[3] = rk; p[4] = rl;
    p[5] = (uint32_t)(strand & 3) << 30;            /* type 0 */
    p[8] = (uint32_t)score;
#endif
}

static bw_t hit_k(const uint32_t *p)
{
#ifdef OR_WIDE
    return (uint64_t)p[2] | (uint64_t)p[3] << 32;
#else
    return p[1];
#endif
}

static bw_t hit_l(const uint32_t *p)
{
#ifdef OR_WIDE
    return (uint64_t)p[4] | (uint64_t)p[5] << 32;
#else
    return p[2];
#endif
}

/* bwt_match_gap (bwtgap.c:118-331).  width/width_seed are 2*(len+1) word arrays. */
static void match_gap(or_index_t *ix, stack_t_ *st, const or_opt_t *opt, const uint8_t *seq, int len,
                      int strand, bw_t *width, const bw_t *width_seed, hitv_t *out,
                      uint64_t *pops)
{
    int best_score = SCORE(opt, opt->max_diff + 1, opt->max_gapo + 1, opt->max_gape + 1);
    int best_diff = opt->max_diff + 1, max_diff = opt->max_diff;
    cnt_t best_cnt = 0;
    int n_aln = 0;
    const bw_t T = ix->f.T;
    out->n = 0;
    stack_reset(st);
    push(st, len, 0, T, 0, T, 0, 0, 0, 0, 0, opt);
#ifdef OR_DUP_STATS
    /* the search's expanded nodes: (i, k, l, rk, state) -> counts, open addressing */
    enum { DUPCAP = 1 << 18 };
    typedef struct { uint64_t key, key2; uint32_t cnt; uint32_t used; } dupe_t;
    static __thread dupe_t *dtab;
    if (!dtab) dtab = (dupe_t *)calloc(DUPCAP, sizeof(dupe_t));
    else memset(dtab, 0, sizeof(dupe_t) * DUPCAP);
    uint64_t d_exp = 0, d_ex = 0, d_dom = 0;
#endif
    while (st->n_entries) {
        ent_t e;
        int i, m, m_seed = 0, hit = 0, allow_diff, allow_M, tmp;
        bw_t k, l, rk, rl, sk[4], sl[4], srk[4], srl[4], occ;
        if (st->n_entries > opt->max_entries) break;
        pop(st, &e);
        if (pops) ++*pops;
        k = e.k; l = e.l; rk = e.rk; rl = e.rl;
        i = (int)(e.info & 0xffff);
        if (!(opt->mode & MODE_NONSTOP) && (int)(e.info >> 21) > best_score + opt->s_mm) break;
        m = max_diff - (e.n_mm + e.n_gapo);
        if (opt->mode & MODE_GAPE) m -= e.n_gape;
        if (m < 0) continue;
        if (width_seed) {
            m_seed = opt->max_seed_diff - (e.n_mm + e.n_gapo);
            if (opt->mode & MODE_GAPE) m_seed -= e.n_gape;
        }
        if (i > 0 && m < (int)width[2 * (i - 1) + 1]) continue;
        if (i == 0) hit = 1;
        else if (m == 0 && (e.state == ST_M || (opt->mode & MODE_GAPE) || e.n_gape == opt->max_gape)) {
            HIST_DEPTH(len - i);
            if (match_exact(ix, seq, i, &k, &l, &rk, &rl)) hit = 1;
            else continue;
        }
        if (hit) {
            int score = SCORE(opt, e.n_mm, e.n_gapo, e.n_gape);
            int do_add = 1;
            if (n_aln == 0) {
                best_score = score;
                best_diff = e.n_mm + e.n_gapo;
                if (opt->mode & MODE_GAPE) best_diff += e.n_gape;
                if (!(opt->mode & MODE_NONSTOP))
                    max_diff = (best_diff + 1 > opt->max_diff) ? opt->max_diff : best_diff + 1;
            }
            if (score == best_score) best_cnt += (cnt_t)(l - k + 1);
            else if (best_cnt > opt->max_top2) break;
            if (e.n_gapo) {
                int j;
                for (j = 0; j != n_aln; ++j)
                    if (hit_k(out->a + HW * j) == k && hit_l(out->a + HW * j) == l) break;
                if (j < n_aln) do_add = 0;
            }
            if (do_add) {
                shadow(l - k + 1, T, e.last_diff_pos, width);
                if (out->n == out->m) {
                    out->m = out->m ? out->m * 2 : 16;
                    out->a = (uint32_t *)realloc(out->a, sizeof(uint32_t) * HW * out->m);
                }
                put_hit(out->a + HW * out->n, &e, k, l, rk, rl, strand, score);
                ++out->n; ++n_aln;
            }
            continue;
        }
#ifdef OR_DUP_STATS
        {
            const uint64_t key = (uint64_t)k << 32 | (uint64_t)l, key2 = (uint64_t)rk << 32 | (uint64_t)i << 4 | e.state;
            const uint32_t cnt = (uint32_t)e.n_mm | (uint32_t)e.n_gapo << 8 | (uint32_t)e.n_gape << 16;
            uint64_t h = (key * 0x9E3779B97F4A7C15ull) ^ (key2 * 0xC2B2AE3D27D4EB4Full);
            int exact = 0, dom = 0;
            /* every earlier expansion of this node (several count triples may share it) */
            for (uint32_t j = (uint32_t)(h >> 46) & (DUPCAP - 1); dtab[j].used; j = (j + 1) & (DUPCAP - 1)) {
                if (dtab[j].key != key || dtab[j].key2 != key2) continue;
                const uint32_t c = dtab[j].cnt;
                if (c == cnt) exact = 1;
                else if ((c & 255) <= (cnt & 255) && ((c >> 8) & 255) <= ((cnt >> 8) & 255) && (c >> 16) <= (cnt >> 16))
                    dom = 1;
            }
            ++d_exp;
            if (exact) ++d_ex;
            else if (dom) ++d_dom;
            if (!exact && d_exp < DUPCAP / 2) {
                uint32_t j = (uint32_t)(h >> 46) & (DUPCAP - 1);
                while (dtab[j].used) j = (j + 1) & (DUPCAP - 1);
                dtab[j].key = key; dtab[j].key2 = key2; dtab[j].cnt = cnt; dtab[j].used = 1;
            }
        }
#endif
        --i;
        HIST_DEPTH(len - i);
        step_all(ix, k, l, rk, rl, sk, sl, srk, srl);
        occ = l - k + 1;
        allow_diff = allow_M = 1;
        if (i > 0) {
            int ii = i - (len - opt->seed_len);
            if ((int)width[2 * (i - 1) + 1] > m - 1) allow_diff = 0;
            else if ((int)width[2 * (i - 1) + 1] == m - 1 && (int)width[2 * i + 1] == m - 1 &&
                     width[2 * (i - 1)] == width[2 * i]) allow_M = 0;
            if (width_seed && ii > 0) {
                if ((int)width_seed[2 * (ii - 1) + 1] > m_seed - 1) allow_diff = 0;
                else if ((int)width_seed[2 * (ii - 1) + 1] == m_seed - 1 && (int)width_seed[2 * ii + 1] == m_seed - 1 &&
                         width_seed[2 * (ii - 1)] == width_seed[2 * ii]) allow_M = 0;
            }
        }
        tmp = (opt->mode & MODE_LOGGAP) ? int_log2(e.n_gape + e.n_gapo) / 2 + 1 : e.n_gapo + e.n_gape;
        if (allow_diff && i >= opt->indel_end_skip + tmp && len - i >= opt->indel_end_skip + tmp) {
            if (e.state == ST_M) {
                if (e.n_gapo < opt->max_gapo) {
                    push(st, i, k, l, rk, rl, e.n_mm, e.n_gapo + 1, e.n_gape, ST_I, 1, opt);
                    for (int j = 0; j != 4; ++j)
                        if (sk[j] <= sl[j])
                            push(st, i + 1, sk[j], sl[j], srk[j], srl[j], e.n_mm, e.n_gapo + 1, e.n_gape, ST_D, 1, opt);
                }
            } else if (e.state == ST_I) {
                if (e.n_gape < opt->max_gape)
                    push(st, i, k, l, rk, rl, e.n_mm, e.n_gapo, e.n_gape + 1, ST_I, 1, opt);
            } else if (e.state == ST_D) {
                if (e.n_gape < opt->max_gape) {
                    if (e.n_gape + e.n_gapo < max_diff || occ < (bw_t)opt->max_del_occ) {
                        for (int j = 0; j != 4; ++j)
                            if (sk[j] <= sl[j])
                                push(st, i + 1, sk[j], sl[j], srk[j], srl[j], e.n_mm, e.n_gapo, e.n_gape + 1, ST_D, 1, opt);
                    }
                }
            }
        }
        if (allow_diff && allow_M) {
            for (int j = 1; j <= 4; ++j) {
                int c = (seq[i] + j) & 3;
                int is_mm = (j != 4 || seq[i] > 3);
                if (sk[c] <= sl[c])
                    push(st, i, sk[c], sl[c], srk[c], srl[c], e.n_mm + is_mm, e.n_gapo, e.n_gape, ST_M, is_mm, opt);
            }
        } else if (seq[i] < 4) {
            int c = seq[i] & 3;
            if (sk[c] <= sl[c])
                push(st, i, sk[c], sl[c], srk[c], srl[c], e.n_mm, e.n_gapo, e.n_gape, ST_M, 0, opt);
        }
    }
#ifdef OR_DUP_STATS
    {
        const int o = n_aln > 0 ? 0 : 3;
        tl_dup[o] += d_exp; tl_dup[o + 1] += d_ex; tl_dup[o + 2] += d_dom;
    }
#endif
}

/* bwt_match_gap (bwtgap.c:118-331) called directly, as bwt_splice_match does
 * (bwtgap.c:812, :919, :1192): the caller's widths, mutated in place by gap_shadow
 * (Q6); seed 0 = width_seed NULL, 1 = its own array, 2 = aliased to width
 * (bwtgap.c:809).  The stack has the caller's n_stacks (aux->stack). */
int OR(match_gap)(const or_index_t *cix, const or_opt_t *opt, int n_stacks, const uint8_t *seq, int len, int strand,
                  bw_t *width, int seed, const bw_t *width_seed, uint32_t **hits)
{
    or_index_t *ix = (or_index_t *)cix;
    stack_t_ *st = stack_new(n_stacks);
    hitv_t hv = {0, 0, NULL};
    const bw_t *ws = seed == 2 ? width : seed == 1 ? width_seed : NULL;
    match_gap(ix, st, opt, seq, len, strand, width, ws, &hv, NULL);
    stack_del(st);
    *hits = hv.a ? hv.a : (uint32_t *)calloc(HW, sizeof(uint32_t));
    return hv.n;
}

static void revcomp(int len, const uint8_t *s, uint8_t *d)   /* seq_reverse(.., 1), bwaseqio.c:73-84 */
{
    for (int i = 0; i < len; ++i) {
        uint8_t c = s[len - 1 - i];
        d[i] = c < 4 ? (uint8_t)(3 - c) : c;
    }
}

/* bwa_cal_sa_reg_gap (bwtaln.c:246-417).  `opt` is the caller's option block and
 * is mutated exactly as the reference mutates it through aux->opt. */
long OR(cal_sa_reg_gap)(const or_index_t *cix, int n, const uint32_t *lens, const uint8_t *codes,
                       or_opt_t *opt, int32_t *n_aln, uint32_t *flags, uint32_t **hits_out,
                       uint64_t *stats)
{
    or_index_t *ix = (or_index_t *)cix;
    or_opt_t local = *opt;                 /* :254, copied before the GAPE clear */
    or_opt_t *cur = opt;                   /* aux->opt (:259) */
    int max_len = 0;
    uint64_t pops = 0, q0 = tl_queries;
    opt->mode &= ~MODE_GAPE;               /* :261 */
    for (int i = 0; i < n; ++i) if ((int)lens[i] > max_len) max_len = (int)lens[i];
    if (opt->fnr > 0.0) local.max_diff = OR(cal_maxdiff)(max_len, 0.02, opt->fnr);
    if (local.max_diff < local.max_gapo) local.max_gapo = local.max_diff;
    stack_t_ *st = stack_new(SCORE(&local, local.max_diff + 1, local.max_gapo + 1, local.max_gape + 1));
    bw_t *wb = (bw_t *)calloc(2 * (max_len + 1), sizeof(bw_t));
    bw_t *ws = (bw_t *)calloc(2 * (max_len + 1), sizeof(bw_t));
    uint8_t *rc = (uint8_t *)calloc(max_len + 1, 1);
    hitv_t hv = {0, 0, NULL}, all = {0, 0, NULL};
    size_t off = 0;
    for (int r = 0; r < n; ++r) {
        const uint8_t *seq = codes + off;
        int len = (int)lens[r];
        off += lens[r];
        n_aln[r] = 0;
        flags[r] = 0;
        int nN = 0;
        for (int j = 0; j < len; ++j) if (seq[j] > 3) ++nN;
        if (nN > local.max_diff) { flags[r] = 2; continue; }          /* :314-317 */
        if (len >= 15) {                                               /* :324-325 (memcmp of 15) */
            int a = 1, t = 1;
            for (int j = 0; j < 15; ++j) { a &= seq[j] == 0; t &= seq[j] == 3; }
            if (a || t) continue;
        }
        if (opt->fnr > 0.0) cur->max_diff = OR(cal_maxdiff)(len, 0.02, opt->fnr);   /* :330-331 */
        cur->seed_len = opt->seed_len < len ? opt->seed_len : 0x7fffffff;          /* :332 */
        revcomp(len, seq, rc);
        int found = 0;
        for (int s = 1; s >= 0; --s) {                                 /* :343 rc first */
            const uint8_t *sq = s ? rc : seq;
            int has_seed = len > cur->seed_len;
            if (has_seed) cal_width(ix, opt->seed_len, sq + (len - cur->seed_len), ws);
            else if (cur->max_diff > 0) {
                fprintf(stderr, "oracle: read %d len %d <= seed_len: undefined in the reference (Q5)\n", r, len);
            }
            cal_width(ix, len, sq, wb);
            match_gap(ix, st, cur, sq, len, s, wb, has_seed ? ws : NULL, &hv, &pops);
            if (hv.n) { found = hv.n; break; }
        }
        if (!found) {                                                  /* :362-369 */
            flags[r] |= 1;
            cur = &local;
            continue;
        }
        hv.a[H_START] = 0; hv.a[H_END] = (uint32_t)(len - 1);         /* :371-372 */
        n_aln[r] = found;
        if (all.n + found > all.m) {
            all.m = (all.n + found) * 2 + 16;
            all.a = (uint32_t *)realloc(all.a, sizeof(uint32_t) * HW * all.m);
        }
        memcpy(all.a + HW * all.n, hv.a, sizeof(uint32_t) * HW * found);
        all.n += found;
    }
    free(wb); free(ws); free(rc); free(hv.a);
    stack_del(st);
    if (stats) { stats[0] = tl_queries - q0; stats[1] = pops; }
    *hits_out = all.a ? all.a : (uint32_t *)calloc(HW, sizeof(uint32_t));
    return all.n;
}

#ifndef OR_WIDE   /* the splice path's seed extension: 32-bit only, as the reference */
/* BWTAllSARangesForward_Bidirection (2BWT-Interface.c:274-304): the rank queries on
 * the REVERSE BWT at rev_k and rev_l + 1, the FORWARD C table. */
static void step_all_fwd(or_index_t *ix, bw_t k, bw_t l, bw_t rk, bw_t rl, bw_t ok[4], bw_t ol[4], bw_t ork[4],
                         bw_t orl[4])
{
    bw_t oL[4], oR[4], oC[4];
    (void)k;
    occ4(&ix->r, rk, oL);
    occ4(&ix->r, rl + 1, oR);
    tl_queries += 2;
    oC[3] = 0;
    for (int c = 2; c >= 0; --c) oC[c] = oC[c + 1] + oR[c + 1] - oL[c + 1];
    for (int c = 0; c < 4; ++c) {
        ork[c] = ix->f.C[c] + oL[c] + 1;
        orl[c] = ix->f.C[c] + oR[c];
        ol[c] = l - oC[c];
        ok[c] = ol[c] - (orl[c] - ork[c]);
    }
}

/* The extension's view of the read: the strand sequence and the direction's width
 * bids at read positions [lo, lo + n).  Any access outside is a restatement error. */
typedef struct { const uint8_t *seq; const int32_t *bid; int lo, n; } ext_win_t;

static uint8_t win_seq(const ext_win_t *w, int p)
{
    if (p < w->lo || p >= w->lo + w->n) { fprintf(stderr, "oracle: extension reads position %d outside [%d, %d)\n", p, w->lo, w->lo + w->n); abort(); }
    return w->seq[p - w->lo];
}

static int win_bid(const ext_win_t *w, int p)
{
    if (p < w->lo || p >= w->lo + w->n) { fprintf(stderr, "oracle: extension reads width %d outside [%d, %d)\n", p, w->lo, w->lo + w->n); abort(); }
    return w->bid[p - w->lo];
}

/* bwt_extend_exact (2BWT-Interface.c:394-439): the outputs change only on a step that
 * keeps the interval non-empty.  Backward consumes *leav; forward never decrements it
 * (:422-436) and extends by the same character until the interval empties. */
static void extend_exact(or_index_t *ix, const ext_win_t *w, int start, int *leav, int type, bw_t *sk, bw_t *sl,
                         bw_t *srk, bw_t *srl)
{
    bw_t k = *sk, l = *sl, rk = *srk, rl = *srl;
    if (type == 1) {
        start -= *leav;
        while (*leav != 0) {
            const uint8_t c = win_seq(w, start + *leav);
            if (c > 3) break;
            step1(ix, c, &k, &l, &rk, &rl);
            if (k > l) break;
            *sk = k; *sl = l; *srk = rk; *srl = rl;
            --*leav;
        }
    } else {
        start += *leav;
        while (*leav != 0) {
            const uint8_t c = win_seq(w, start - *leav);
            if (c > 3) break;
            bw_t ok[4], ol[4], ork[4], orl[4];
            step_all_fwd(ix, k, l, rk, rl, ok, ol, ork, orl);   /* BWTSARangeForward_Bidirection */
            k = ok[c]; l = ol[c]; rk = ork[c]; rl = orl[c];
            if (k > l) break;
            *sk = k; *sl = l; *srk = rk; *srl = rl;
        }
    }
}

/* bwt_extend_backward / bwt_extend_foreward (bwtgap.c:640-663): the stack reset, the
 * seed's entry (i = len, state M, is_diff 0), then bwt_backtracing_search
 * (bwtgap.c:346-511).  aln: the 9 words of the bwt_aln1_t, updated in place;
 * *max_pos in/out; returns 1, 2 or -1.  The gap entry's info word is the reference's
 * score << 21 | i in 32 bits, so a negative len gives a score field of 2047 (the
 * search stops at its first pop unless NONSTOP). */
int or_extend(const or_index_t *cix, const or_opt_t *opt, int n_stacks, int is_backward, int len, const uint8_t *seq,
              const int32_t *bid, int lo, int n, uint32_t *aln, int *max_pos_io)
{
    or_index_t *ix = (or_index_t *)cix;
    const ext_win_t w = {seq, bid, lo, n};
    stack_t_ *st = stack_new(n_stacks);
    stack_reset(st);
    const int a_mm = (int)(aln[0] & 0xFFFF), a_go = (int)((aln[0] >> 16) & 0xFF), a_ge = (int)(aln[0] >> 24);
    push(st, len, aln[1], aln[2], aln[3], aln[4], a_mm, a_go, a_ge, ST_M, 0, opt);
    const int best_score = SCORE(opt, opt->max_diff + 1, opt->max_gapo + 1, opt->max_gape + 1);
    const int max_diff = opt->max_diff;
    const int start = (int)aln[6], end = (int)aln[7];
    int max_pos = *max_pos_io, ret = 0;
    while (st->n_entries != 0) {
        if (st->n_entries > opt->max_entries) break;
        ent_t e;
        pop(st, &e);
        bw_t k = e.k, l = e.l, rk = e.rk, rl = e.rl;
        int i = (int)(e.info & 0xffff);
        if (!(opt->mode & MODE_NONSTOP) && (int)(e.info >> 21) > best_score + opt->s_mm) break;
        int m = max_diff - (e.n_mm + e.n_gapo);
        if (opt->mode & MODE_GAPE) m -= e.n_gape;
        if (m <= 0 || i == 0) {
            if (m == 0 && i != 0)
                extend_exact(ix, &w, is_backward == 0 ? end + len - i + 1 : start - len + i - 1, &i, is_backward,
                             &k, &l, &rk, &rl);
            if (is_backward == 1 && max_pos >= start + i - len && (int)aln[6] > start + i - len) {
                aln[6] = (uint32_t)(start + i - len);
                max_pos = (int)aln[6];
            } else if (is_backward == 0 && max_pos <= end + len - i && (int)aln[7] < end + len - i) {
                aln[7] = (uint32_t)(end + len - i);
                max_pos = (int)aln[7];
            } else {
                continue;
            }
            aln[1] = k; aln[2] = l; aln[3] = rk; aln[4] = rl;
            aln[5] = (aln[5] & 0xC0000000u) | 4u;                       /* BWA_TYPE_SPLICING, strand kept */
            aln[0] = (uint32_t)e.n_mm | (uint32_t)e.n_gapo << 16 | (uint32_t)e.n_gape << 24;
            aln[8] = e.info >> 21;
            if (i == 0) { ret = 1; break; }
            continue;
        }
        --i;
        const int real_pos = is_backward == 1 ? start - len + i : len + end - i;
        bw_t ok[4], ol[4], ork[4], orl[4];
        if (is_backward == 1) step_all(ix, k, l, rk, rl, ok, ol, ork, orl);
        else step_all_fwd(ix, k, l, rk, rl, ok, ol, ork, orl);
        const bw_t occ = l - k + 1;
        int allow_diff = 1;
        if (is_backward == 1 && max_pos < real_pos) {
            const int d = win_bid(&w, real_pos) - win_bid(&w, max_pos);
            if (d > m || (d == m && win_bid(&w, max_pos) != win_bid(&w, max_pos + 1))) allow_diff = 0;
        }
        if (is_backward == 0 && max_pos > real_pos) {
            const int d = win_bid(&w, real_pos) - win_bid(&w, max_pos);
            if (d > m || (d == m && win_bid(&w, max_pos) != win_bid(&w, max_pos - 1))) allow_diff = 0;
        }
        const int tmp = (opt->mode & MODE_LOGGAP) ? int_log2((uint32_t)(e.n_gape + e.n_gapo)) / 2 + 1
                                                  : e.n_gapo + e.n_gape;
        if (allow_diff && i >= opt->indel_end_skip + tmp && len - i >= opt->indel_end_skip + tmp) {
            if (e.state == ST_M) {
                if (e.n_gapo < opt->max_gapo) {
                    push(st, i, k, l, rk, rl, e.n_mm, e.n_gapo + 1, e.n_gape, ST_I, 1, opt);
                    for (int j = 0; j != 4; ++j)
                        if ((is_backward == 1 && ok[j] <= ol[j]) || (is_backward == 0 && ork[j] <= orl[j]))
                            push(st, i + 1, ok[j], ol[j], ork[j], orl[j], e.n_mm, e.n_gapo + 1, e.n_gape, ST_D, 1, opt);
                }
            } else if (e.state == ST_I) {
                if (e.n_gape < opt->max_gape) push(st, i, k, l, rk, rl, e.n_mm, e.n_gapo, e.n_gape + 1, ST_I, 1, opt);
            } else if (e.state == ST_D) {
                if (e.n_gape < opt->max_gape && (e.n_gape + e.n_gapo < max_diff || occ < (bw_t)opt->max_del_occ))
                    for (int j = 0; j != 4; ++j)
                        if (ok[j] <= ol[j])
                            push(st, i + 1, ok[j], ol[j], ork[j], orl[j], e.n_mm, e.n_gapo, e.n_gape + 1, ST_D, 1, opt);
            }
        }
        if (allow_diff == 1) {
            const uint8_t sc = win_seq(&w, real_pos);
            for (int j = 1; j <= 4; ++j) {
                const int c = (sc + j) & 3, is_mm = (j != 4 || sc > 3);
                if ((is_backward == 1 && ok[c] <= ol[c]) || (is_backward == 0 && ork[c] <= orl[c]))
                    push(st, i, ok[c], ol[c], ork[c], orl[c], e.n_mm + is_mm, e.n_gapo, e.n_gape, ST_M, is_mm, opt);
            }
        }
    }
    stack_del(st);
    if (ret == 1) { *max_pos_io = max_pos; return 1; }
    if (*max_pos_io != max_pos) { *max_pos_io = max_pos; return 2; }
    return -1;
}
#endif
