// hsa_splice.hip -- the splice path on the device: bwt_splice_match
// (bwtgap.c:748-1332) for every fallback read of a batch in one persistent kernel.
//
// A read the main search leaves without a hit goes through a long, branchy, sequential
// procedure: six seed searches, a correlation of the seeds' positions, a motif scan of
// the reference between the seeds, then rounds of seed extensions toward each candidate
// splice site with correlations and intron-end checks between them.  The searches it
// can make before its first extension are determined by the read alone and come from the
// batch's prefetch pass (hsa_splice_prefetch_batch, hsa_search.hip): width rows, the six
// seeds, the 12-mer anchors.  Everything after that runs here, one lane per read:
//
// * the control flow of bwt_splice_match is a resumable state machine (sp_ctrl, a
//   switch over resume points): it runs until the read needs a seed extension or is
//   done;
// * the extension (bwt_extend_backward / _foreward -> bwt_backtracing_search,
//   bwtgap.c:346-663) runs in the kernel's main loop, at ONE place for every lane of the
//   wave, a few pops per lane per iteration -- the same search as k_extend
//   (hsa_extend.hip): a bucketed LIFO per lane (heads and counts in LDS, 32-byte
//   entries in an HBM pool with a free list), the entry pushed last kept in registers;
// * bwt_aln_corelate_check (:669-742) and check_site_by_intron_end (:602-635) take their
//   SA -> position lookups on the device (hsa_sa.h); splice_site_search_from_pos
//   (:523-594) reads the packed reference the host's HSP holds (hsa_index_set_text).
//
// Reads whose path the reference leaves undefined here (a read position outside the
// read, a rank position past the text, a text position past the packed array, an SA
// position in no chromosome block), or that outgrow the kernel's per-lane stack, or whose
// prefetched searches did not finish, are not answered: their status tells the caller to
// run the host's own bwt_splice_match for them (bwtaln_gpu.c), so the answers never
// depend on the kernel's capacities.
//
// bwt_array_insert and bwt_find_split_pos_by_record return at their first line
// (bwt_array.c:34, :77): the splice-site record is inert and not kept here.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsa_device.h"
#include "hsa_internal.h"
#include "hsa_sa.h"

#define SP_NT 64                 // lanes per workgroup
#define SP_NIL 0xFFFFu           // empty bucket / free list (16-bit slot numbers)
#ifndef HSA_SP_BUDGET
#define HSA_SP_BUDGET 16         // extension pops per lane per pass of the main loop
#endif
#define SP_POS_MAX 100           // bwt_aln_corelate_check: <= 10 hits x 10 positions (bwtgap.c:684-706)
#define MODE_GAPE 0x01
#define MODE_LOGGAP 0x04
#define MODE_NONSTOP 0x10
#define ST_M 0
#define ST_I 1
#define ST_D 2

// resume points of sp_ctrl
enum {
    PC_START = 0, PC_M3, PC_M5, PC_M6,
    PC_M3_E1, PC_M3_L1, PC_M3_L2, PC_M3_F1, PC_M3_F2,
    PC_M5_L1, PC_M5_L2, PC_M5_F1, PC_M5_F2,
    PC_M6_E0, PC_M6_L1, PC_M6_L2, PC_M6_F1, PC_M6_F2
};
enum { SP_AGAIN = 0, SP_EXT = 1, SP_DONE = 2 };

// splice_site_search_from_pos's motifs (bwtgap.c:533-534): positive GT-AG GC-AG AT-AC,
// negative CT-AC CT-GC GT-AT
__constant__ uint8_t c_motif[2][12] = {{2, 3, 0, 2, 2, 1, 0, 2, 0, 3, 0, 1}, {1, 3, 0, 1, 1, 3, 2, 1, 2, 3, 0, 3}};

// One of bwt_splice_match's bwt_seed_aln_t (q, q + 1, q + 2 of the chosen strand): its hit
// count, its hit list in the prefetch's hit arrays, and aln[0] as the reference's code
// leaves it (extensions, memcpy's and reductions rewrite aln[0] only).
struct SpSlot {
    int32_t n;
    int32_t kind;                // 0..2 seed t (bwtgap.c:816-819 sets every hit's start/end), 3 an anchor
    uint64_t list;               // record index of the first hit
    uint32_t a0[9];
};

// A lane's state between resume points (global memory: read only at control steps).
struct SpLane {
    int32_t pc, read, L, sl, strand, mt, nsite, m, motif, bmap, n_out, max_pos, ext_ret, gape, anchor6, xl, xdir;
    int32_t status;
    uint32_t seq_pos;
    uint32_t n_ext, n_sa;
    SpSlot A, B, C;              // q, q + 1, q + 2
    uint32_t res0[9], res1[9];   // res_aln[0], res_aln[1] (calloc'd, bwtgap.c:854)
};

struct SpArgs {
    RankDir fwd, rev;
    uint32_t T, rT;
    uint32_t C[4];
    SaView sav;
    const uint32_t *text;        // the HSP's packedDNA words
    uint64_t text_chars;         // characters the allocated words hold
    uint32_t dna_len;
    PfDev pf;
    hsa_regime_t rg;             // the extension regime; max_diff per read from pf.amd
    uint32_t nb, cap, site_cap, ref_cap, lbuf_words;
    // score -> bucket over the scores an extension can reach (dense, in score order;
    // 0xff: none -- a push there is handed back as HSA_SP_SCORE)
    uint8_t bmap[HSA_SP_MAX_STACKS];
    uint4 *pool;                 // per lane: cap entries x 2 uint4
    SpLane *lanes;
    uint32_t *lbuf;              // per lane: positions (3 x SP_POS_MAX) | sites | reference bytes
    unsigned long long *next;    // the read queue's head
    unsigned long long *ctr;     // [0] extensions [1] pops [2] SA lookups [3] reads not answered
    uint32_t *res;               // HSA_SP_RES_WORDS per read
};

__device__ __forceinline__ uint32_t sp_char(const SpArgs &a, uint32_t k)   // packedDNA[k>>4] >> ((~k & 15) << 1) & 3
{
    return (a.text[k >> 4] >> ((~k & 15u) << 1)) & 3u;
}

__device__ __forceinline__ void sp_copy(uint32_t *d, const uint32_t *s)
{
#pragma unroll
    for (int w = 0; w < 9; ++w) d[w] = s[w];
}

// aln->type = BWA_TYPE_SPLICING (bwtaln.h: type:30, strand:2 in word 5)
__device__ __forceinline__ void sp_splicing(uint32_t *x) { x[5] = (x[5] & 0xC0000000u) | 4u; }

// Word w of the slot's hit i.
__device__ uint32_t sp_word(const SpArgs &a, const SpLane &S, const SpSlot &Q, int i, int w)
{
    if (i == 0) return Q.a0[w];
    if (Q.kind < 3 && (w == 6 || w == 7)) {
        const int st = Q.kind * S.sl, la = S.sl + (Q.kind == 2 ? S.L % 3 : 0);
        return (uint32_t)(w == 6 ? st : st + la - 1);
    }
    const uint32_t *h = (Q.kind < 3 ? a.pf.hits_s : a.pf.hits_a) + (Q.list + (uint64_t)i) * 9u;
    return h[w];
}

// p->n_aln = 1, p->aln = a copy of hit i (bwtgap.c:729-734)
__device__ void sp_take(const SpArgs &a, const SpLane &S, SpSlot &Q, int i)
{
    if (i != 0) {
        uint32_t t[9];
#pragma unroll
        for (int w = 0; w < 9; ++w) t[w] = sp_word(a, S, Q, i, w);
        sp_copy(Q.a0, t);
    }
    Q.n = 1;
}

// seed t of strand s (bwtgap.c:797-820)
__device__ void sp_seed_slot(const SpArgs &a, SpLane &S, SpSlot &Q, int r, int s, int t)
{
    const size_t c = 8 * (size_t)r + 3 * s + t;
    Q.n = a.pf.call_n[c];
    Q.kind = t;
    Q.list = a.pf.call_hit[c];
#pragma unroll
    for (int w = 0; w < 9; ++w) Q.a0[w] = 0;
    if (Q.n > 0) {
        const uint32_t *h = a.pf.hits_s + Q.list * 9u;
#pragma unroll
        for (int w = 0; w < 9; ++w) Q.a0[w] = h[w];
        const int la = S.sl + (t == 2 ? S.L % 3 : 0);
        Q.a0[6] = (uint32_t)(t * S.sl);
        Q.a0[7] = (uint32_t)(t * S.sl + la - 1);
    }
}

// the 12-mer anchor of the chosen strand (bwtgap.c:910-928, :1187-1201): a new hit list;
// aln[0]'s start / end set when it has hits
__device__ void sp_anchor_slot(const SpArgs &a, SpLane &S, SpSlot &Q, int r, int start, int end)
{
    const size_t c = 8 * (size_t)r + 6 + S.strand;
    if (a.pf.call_n[c] < 0) { S.status = HSA_SP_CALL; return; }     // not searched: cannot happen
    if (a.pf.call_fl[c] & HSA_F_OVERFLOW) { S.status = HSA_SP_CALL; return; }
    Q.n = a.pf.call_n[c];
    Q.kind = 3;
    Q.list = a.pf.call_hit[c];
#pragma unroll
    for (int w = 0; w < 9; ++w) Q.a0[w] = 0;
    if (Q.n > 0) {
        const uint32_t *h = a.pf.hits_a + Q.list * 9u;
#pragma unroll
        for (int w = 0; w < 9; ++w) Q.a0[w] = h[w];
        Q.a0[6] = (uint32_t)start;
        Q.a0[7] = (uint32_t)end;
    }
}

// BWTRetrievePositionFromSAIndex (2BWT-Interface.c:329-361): occ always, the block's
// sequence id only when a block holds it (else the reference leaves the caller's stale
// variable: not answered here)
__device__ __forceinline__ bool sp_sa(const SpArgs &a, SpLane &S, uint32_t j, uint32_t &sid, uint32_t &occ)
{
    uint32_t ori = 0;
    occ = hsa_sa_value(a.sav, j);
    ++S.n_sa;
    if (!hsa_sa_block(a.sav, occ, sid, ori)) { S.status = HSA_SP_SA; return false; }
    return true;
}

// bwt_aln_corelate_check (bwtgap.c:669-742): the nearest pair (50 < distance < 50 000 on
// one sequence) between the first 10 positions of P's first 10 hits and the first 50 of
// every Q hit; on success P and Q keep that pair's hits only.  Returns P's position, or
// 0xffffffff.
__device__ uint32_t sp_corr(const SpArgs &a, SpLane &S, SpSlot &P, SpSlot &Q, uint32_t *pos)
{
    int tot = 0, cur = 0;
    for (int i = 0; i < P.n && i < 10; ++i) {
        const uint32_t k = sp_word(a, S, P, i, 1), l = sp_word(a, S, P, i, 2);
        const uint32_t w = l - k + 1u;
        tot += (int)(w > 10u ? 10u : w);
        const uint32_t lim = k + 10u;
        for (uint32_t j = k; j <= l && j < lim; ++j) {
            if (cur >= SP_POS_MAX) { S.status = HSA_SP_LOOP; return 0xffffffffu; }
            uint32_t sid = 0, occ = 0;
            if (!sp_sa(a, S, j, sid, occ)) return 0xffffffffu;
            pos[3 * cur] = sid;
            pos[3 * cur + 1] = occ;
            pos[3 * cur + 2] = (uint32_t)i;
            ++cur;
        }
    }
    if (tot != cur) { S.status = HSA_SP_LOOP; return 0xffffffffu; }   // the reference would read unset entries
    uint32_t min_dist = 0xffffffffu, res_pos = 0xffffffffu;
    int t1 = 0, t2 = 0;
    for (int i = 0; i < Q.n; ++i) {
        const uint32_t k = sp_word(a, S, Q, i, 1), l = sp_word(a, S, Q, i, 2);
        if (l == 0xffffffffu) { S.status = HSA_SP_LOOP; return 0xffffffffu; }
        const uint32_t lim = k + 50u;
        for (uint32_t j = k; j <= l && j < lim; ++j) {
            uint32_t sid = 0, occ = 0;
            if (!sp_sa(a, S, j, sid, occ)) return 0xffffffffu;
            for (int x = 0; x < tot; ++x) {
                const int dist = (int)(occ - pos[3 * x + 1]);
                if (pos[3 * x] == sid && dist > 50 && dist < 50000 && min_dist > (uint32_t)dist) {
                    min_dist = (uint32_t)dist;
                    res_pos = pos[3 * x + 1];
                    t1 = (int)pos[3 * x + 2];
                    t2 = i;
                }
            }
        }
    }
    if (min_dist != 0xffffffffu) {
        sp_take(a, S, P, t1);
        sp_take(a, S, Q, t2);
    }
    return res_pos;
}

// splice_site_search_from_pos (bwtgap.c:523-594): the read positions in (left, right)
// where the reference after `pos` shows a splice motif of the strand, motif type in the
// top two bits
__device__ void sp_sites(const SpArgs &a, SpLane &S, const uint8_t *seq, int bw, uint32_t pos, int ext, int left,
                         int right, uint32_t *sites, uint8_t *ref)
{
    const int ref_len = right - left - 1;
    S.nsite = 0;
    if (bw == 1) pos -= (uint32_t)ref_len;
    else pos += (uint32_t)(left + 1 + ext);
    if (ref_len <= 0) {
        // calloc of a negative size: the reference's copy loop writes through NULL when it runs
        if (ref_len < 0 && pos < pos + (uint32_t)ref_len && pos < a.dna_len) S.status = HSA_SP_TEXT;
        return;
    }
    if ((uint32_t)ref_len > a.ref_cap) { S.status = HSA_SP_LOOP; return; }
    const uint32_t end = pos + (uint32_t)ref_len;
    int l = 0;
    for (uint32_t k = pos; k < end && k < a.dna_len; ++k) ref[l++] = (uint8_t)sp_char(a, k);
    for (int x = l; x < ref_len; ++x) ref[x] = 0;       // calloc'd
    const uint8_t *mot = c_motif[S.strand];
    for (int i = 0; i < 3; ++i) {
        const uint8_t m0 = mot[4 * i + (bw ? 2 : 0)], m1 = mot[4 * i + (bw ? 3 : 1)];
        for (int j = 2; j < ref_len - 1; ++j) {
            const int rp = bw ? ref_len - 2 - j : j;
            if (ref[rp] != m0 || ref[rp + 1] != m1) continue;
            const int sp = bw ? right - j : left + j;
            if (sp < 0 || sp >= S.L) { S.status = HSA_SP_WIN; return; }
            if ((!bw && ref[rp - 1] == seq[sp]) || (bw && ref[rp + 2] == seq[sp])) {
                if ((uint32_t)S.nsite >= a.site_cap) { S.status = HSA_SP_LOOP; return; }
                sites[S.nsite++] = (uint32_t)i << 30 | (uint32_t)sp;
            }
        }
        if ((!bw && S.strand == 1 && i == 0) || (bw && S.strand == 0 && i == 0)) i += 1;   // :587-589
    }
}

// check_site_by_intron_end (bwtgap.c:602-635): the intron end next to each position of
// the hit against the motif type (0 -> 1 on the strands where they share that end);
// returns the type matched, or 3
__device__ int sp_check_site(const SpArgs &a, SpLane &S, const uint32_t *aln, int bw, int type, int strand)
{
    const uint8_t *mot = c_motif[strand];
    const uint32_t k0 = aln[1], l0 = aln[2], end = aln[7];
    if (l0 == 0xffffffffu) { S.status = HSA_SP_LOOP; return 3; }
    for (uint32_t m = k0; m <= l0; ++m) {
        const uint32_t occ = hsa_sa_value(a.sav, m);
        ++S.n_sa;
        const uint32_t k = bw == 1 ? occ - 2u : occ + end + 1u, k2 = k + 1u;
        if (k >= a.text_chars || k2 >= a.text_chars) { S.status = HSA_SP_TEXT; return 3; }
        const uint32_t r0 = sp_char(a, k), r1 = sp_char(a, k2);
        const int o = bw == 0 ? 0 : 2;
        if (r0 == mot[type * 4 + o] && r1 == mot[type * 4 + o + 1]) return type;
        if (type == 0 && ((bw == 1 && strand == 1) || (bw == 0 && strand == 0))) {
            type = 1;
            if (r0 == mot[4 + o] && r1 == mot[5 + o]) return type;
        }
    }
    return 3;
}

__device__ void sp_skip_motif(SpLane &S, const uint32_t *sites)   // bwtgap.c:947-948 (:1078, :1221)
{
    while (S.m + 1 < S.nsite && (int)(sites[S.m + 1] >> 30) == S.motif) S.m++;
}

__device__ void sp_finish(const SpArgs &a, SpLane &S)
{
    uint32_t *o = a.res + (size_t)(a.pf.idx ? (uint32_t)a.pf.idx[S.read] : (uint32_t)S.read) * HSA_SP_RES_WORDS;
    o[0] = (uint32_t)S.status;
    o[1] = S.status ? 0u : (uint32_t)S.n_out;
#pragma unroll
    for (int w = 0; w < 9; ++w) { o[2 + w] = S.res0[w]; o[11 + w] = S.res1[w]; }
    if (S.status) atomicAdd(a.ctr + 3, 1ull);
    S.read = -1;
}

__device__ void sp_init(const SpArgs &a, SpLane &S, int r)
{
    S.read = r;
    S.pc = PC_START;
    S.L = (int)a.pf.lens[r];
    S.sl = S.L / 3;
    S.strand = 0;
    S.status = 0;
    S.n_out = 0;
    S.bmap = 0;
    S.anchor6 = 0;
    S.nsite = 0;
    S.gape = (a.rg.mode & MODE_GAPE) ? 1 : 0;            // aux_ext->opt: a copy of local_opt (:777-782)
#pragma unroll
    for (int w = 0; w < 9; ++w) { S.res0[w] = 0; S.res1[w] = 0; }
}

// An extension call: direction (0 foreward on A, 1 backward on C), aux_ext->len; resumes
// at LABEL with S.ext_ret, S.max_pos and the slot's aln[0] as the reference leaves them.
#define SP_CALL_EXT(DIR, LEN, LABEL)                                  \
    do {                                                              \
        S.xdir = (DIR);                                               \
        S.xl = (LEN);                                                 \
        S.pc = (LABEL);                                               \
        return SP_EXT;                                                \
        case (LABEL):;                                                \
    } while (0)
#define SP_FINISH()             \
    do {                        \
        sp_finish(a, S);        \
        return SP_DONE;         \
    } while (0)
#define SP_CHECK()                  \
    do {                            \
        if (S.status) SP_FINISH();  \
    } while (0)

// bwt_splice_match (bwtgap.c:748-1332) from the last resume point to the next extension
// call or the end.  Every variable that lives across an extension is in S.
__device__ __noinline__ int sp_ctrl(const SpArgs &a, SpLane &S, uint32_t *lb)
{
    uint32_t *const pos = lb;
    uint32_t *const sites = lb + 3 * SP_POS_MAX;
    uint8_t *const ref = reinterpret_cast<uint8_t *>(sites + a.site_cap);
    const uint8_t *const seq = a.pf.scodes + (size_t)(2 * S.read + S.strand) * a.pf.sc;   // valid once strand is set
    const int r = S.read;
    switch (S.pc) {
    case PC_START: {
        // the six seeds (bwtgap.c:797-848): strand 0's three, their correlation when two
        // or more hit, else strand 1's (seed 2 of strand 0 skipped when 0 and 1 miss)
        int jj = 0, mt = 0;
        uint32_t seq_pos = 0xffffffffu;
        for (int i = 0; i < 6; ++i) {
            const int s = i / 3, t = i % 3;
            const size_t c = 8 * (size_t)r + i;
            if (a.pf.call_fl[c] & HSA_F_OVERFLOW) { S.status = HSA_SP_CALL; SP_FINISH(); }
            if (a.pf.call_n[c] != 0) { ++jj; mt += 1 << t; }
            if (i == 1 && jj == 0) { i += 1; jj = 0; mt = 0; continue; }
            if ((i == 2 || i == 5) && jj > 1) {
                S.strand = s;
                sp_seed_slot(a, S, S.A, r, s, 0);
                sp_seed_slot(a, S, S.B, r, s, 1);
                sp_seed_slot(a, S, S.C, r, s, 2);
                if (mt == 5 || mt == 7) seq_pos = sp_corr(a, S, S.A, S.C, pos);
                else if (mt == 3) seq_pos = sp_corr(a, S, S.A, S.B, pos);
                else if (mt == 6) seq_pos = sp_corr(a, S, S.B, S.C, pos);
                SP_CHECK();
                if (seq_pos != 0xffffffffu) break;
            }
            if (i == 2) { jj = 0; mt = 0; }
        }
        if (jj < 2 || seq_pos == 0xffffffffu) SP_FINISH();   // *_n_aln = 0 (:857-858)
        S.mt = mt;
        S.seq_pos = seq_pos;
        S.pc = mt == 3 ? PC_M3 : mt == 6 ? PC_M6 : PC_M5;
        return SP_AGAIN;
    }

    // ---- seeds 0 and 1 (bwtgap.c:881-1031)
    case PC_M3:
        sp_sites(a, S, seq, 0, S.seq_pos, (int)((S.A.a0[0] >> 16) & 0xFFu) + (int)(S.A.a0[0] >> 24), (int)S.B.a0[7], S.L,
                 sites, ref);
        SP_CHECK();
        S.max_pos = (int)S.B.a0[7];
        SP_CALL_EXT(0, S.max_pos - (int)S.A.a0[7], PC_M3_E1);
        if (S.ext_ret != 1) SP_FINISH();
        S.motif = (int)(sites[0] >> 30) * (S.nsite > 0);
        sp_copy(S.res0, S.A.a0);
        sp_anchor_slot(a, S, S.C, r, S.L - 12, S.L - 1);     // the last 12 bases (:910-928)
        SP_CHECK();
        if (S.C.n == 0) SP_FINISH();
        {
            const uint32_t o1 = sp_corr(a, S, S.A, S.C, pos);
            SP_CHECK();
            if (o1 == 0x3fffffffu) SP_FINISH();
        }
        sp_copy(S.res1, S.C.a0);
        for (S.m = 0; S.m < S.nsite; ++S.m) {
            S.max_pos = (int)(sites[S.m] & 0x3fffffffu);
            if (S.motif != (int)(sites[S.m] >> 30)) {
                sp_copy(S.res0, S.A.a0);
                S.motif = (int)(sites[S.m] >> 30);
            }
            SP_CALL_EXT(0, S.max_pos - (int)S.A.a0[7], PC_M3_L1);
            if (S.ext_ret != 1) { sp_skip_motif(S, sites); continue; }
            S.max_pos += 1;
            S.xl = (int)S.res1[6] - S.max_pos;
            if (S.xl > 0) {
                sp_copy(S.C.a0, S.res1);
                SP_CALL_EXT(1, S.xl, PC_M3_L2);
                if (S.ext_ret != 1) continue;
                S.seq_pos = sp_corr(a, S, S.A, S.C, pos);
                SP_CHECK();
                if (S.seq_pos == 0xffffffffu) continue;
                {
                    const int mtc = sp_check_site(a, S, S.C.a0, 1, S.motif, S.strand);
                    SP_CHECK();
                    if (mtc != 3) { S.n_out = 2; S.bmap = 1; break; }
                }
                continue;
            } else {
                S.n_out = 1;
                S.bmap = 1;
                continue;
            }
        }
        if (S.bmap == 0) {
            sp_copy(S.C.a0, S.res1);
            S.max_pos = (int)S.B.a0[7] + 1;
            SP_CALL_EXT(0, (int)S.C.a0[6] - (int)S.A.a0[7] - 1, PC_M3_F1);
            S.n_out = 1;
            if (S.ext_ret == 2) {
                S.max_pos += 1;
                S.xl = (int)S.C.a0[6] - S.max_pos;
                if (S.xl > 0) {
                    SP_CALL_EXT(1, S.xl, PC_M3_F2);
                    if (S.ext_ret == 1) {
                        S.C.a0[6] = (uint32_t)S.max_pos;
                        S.seq_pos = sp_corr(a, S, S.A, S.C, pos);
                        SP_CHECK();
                        if (S.seq_pos != 0xffffffffu) S.n_out = 2;
                    }
                }
            }
        }
        if (S.n_out != 0) { sp_copy(S.res0, S.A.a0); sp_splicing(S.res0); }
        if (S.n_out == 2) { sp_copy(S.res1, S.C.a0); sp_splicing(S.res1); }
        SP_FINISH();

    // ---- seeds 0 and 2 (and 1) (bwtgap.c:1032-1152)
    case PC_M5:
        sp_sites(a, S, seq, 0, S.seq_pos, (int)((S.A.a0[0] >> 16) & 0xFFu) + (int)(S.A.a0[0] >> 24), (int)S.A.a0[7],
                 (int)S.C.a0[6], sites, ref);
        SP_CHECK();
        S.gape = 0;
        S.motif = (int)(sites[0] >> 30) * (S.nsite > 0);
        sp_copy(S.res0, S.A.a0);
        sp_copy(S.res1, S.C.a0);
        for (S.m = 0; S.m < S.nsite; ++S.m) {
            S.max_pos = (int)(sites[S.m] & 0x3fffffffu);
            if (S.motif != (int)(sites[S.m] >> 30)) {
                sp_copy(S.A.a0, S.res0);
                S.motif = (int)(sites[S.m] >> 30);
            }
            sp_copy(S.C.a0, S.res1);
            SP_CALL_EXT(0, S.max_pos - (int)S.A.a0[7], PC_M5_L1);
            if (S.ext_ret != 1) { sp_skip_motif(S, sites); continue; }
            S.max_pos += 1;
            SP_CALL_EXT(1, (int)S.C.a0[6] - S.max_pos, PC_M5_L2);
            if (S.ext_ret != 1) continue;
            {
                const int mtc = sp_check_site(a, S, S.C.a0, 1, S.motif, S.strand);
                SP_CHECK();
                if (mtc != 3) { S.n_out = 2; S.bmap = 1; break; }
            }
        }
        if (S.bmap == 0) {
            S.gape = 0;
            S.max_pos = (int)S.A.a0[7] + 1;
            SP_CALL_EXT(0, (int)S.C.a0[6] - (int)S.A.a0[7] - 1, PC_M5_F1);
            if (S.ext_ret == -1) {
                S.n_out = 0;
            } else if (S.ext_ret == 1) {
                S.n_out = 2;
            } else {
                S.max_pos = (int)S.A.a0[7] + 1;
                S.gape = 1;
                SP_CALL_EXT(1, (int)S.C.a0[6] - S.max_pos, PC_M5_F2);
                S.seq_pos = sp_corr(a, S, S.A, S.C, pos);
                SP_CHECK();
                S.n_out = (S.ext_ret == -1 || S.seq_pos == 0xffffffffu) ? 0 : 2;
            }
        }
        if (S.n_out != 0) {
            sp_copy(S.res0, S.A.a0);
            sp_copy(S.res1, S.C.a0);
            sp_splicing(S.res0);
            sp_splicing(S.res1);
        }
        SP_FINISH();

    // ---- seeds 1 and 2 (bwtgap.c:1153-1308)
    case PC_M6:
        sp_sites(a, S, seq, 1, S.seq_pos - (uint32_t)S.sl, 0, 0, (int)S.B.a0[6], sites, ref);
        SP_CHECK();
        S.max_pos = (int)S.B.a0[6];
        SP_CALL_EXT(1, (int)S.C.a0[6] - (int)S.B.a0[6], PC_M6_E0);
        if (S.ext_ret != 1) SP_FINISH();
        // the first 12 bases with the whole strand's widths (:1187-1201): its gap_shadow
        // rewrites width_back[0, 12) for the extensions after it
        S.anchor6 = 1;
        sp_anchor_slot(a, S, S.A, r, 0, 11);
        SP_CHECK();
        if (S.A.n == 0) SP_FINISH();
        {
            const uint32_t o1 = sp_corr(a, S, S.A, S.C, pos);
            SP_CHECK();
            if (o1 == 0x3fffffffu) SP_FINISH();
        }
        sp_copy(S.res0, S.A.a0);
        sp_copy(S.res1, S.C.a0);
        S.motif = (int)(sites[0] >> 30) * (S.nsite > 0);
        for (S.m = 0; S.m < S.nsite; ++S.m) {
            S.max_pos = (int)(sites[S.m] & 0x3fffffffu);
            S.xl = (int)S.C.a0[6] - S.max_pos;
            if (S.motif != (int)(sites[S.m] >> 30)) {
                sp_copy(S.C.a0, S.res1);
                S.motif = (int)(sites[S.m] >> 30);
            }
            SP_CALL_EXT(1, S.xl, PC_M6_L1);
            if (S.ext_ret != 1) { sp_skip_motif(S, sites); continue; }
            S.max_pos -= 1;
            S.xl = S.max_pos - (int)S.A.a0[7];
            if (S.xl > 0) {
                sp_copy(S.A.a0, S.res0);
                SP_CALL_EXT(0, S.xl, PC_M6_L2);
                if (S.ext_ret != 1) continue;
                S.seq_pos = sp_corr(a, S, S.A, S.C, pos);
                SP_CHECK();
                if (S.seq_pos == 0xffffffffu) continue;
                {
                    const int mtc = sp_check_site(a, S, S.A.a0, 0, S.motif, S.strand);
                    SP_CHECK();
                    if (mtc != 3) { S.bmap = 1; S.n_out = 2; break; }
                }
                continue;
            } else {
                S.n_out = 1;
                S.bmap = 1;
                break;
            }
        }
        if (S.bmap == 0) {
            S.max_pos = (int)S.C.a0[6] - 1;
            SP_CALL_EXT(1, (int)S.C.a0[6] - (int)S.A.a0[7] - 1, PC_M6_F1);
            if (S.ext_ret == 2) S.n_out = 1;
            S.max_pos -= 1;
            S.xl = S.max_pos - (int)S.A.a0[7];
            if (S.xl > 0) {
                SP_CALL_EXT(0, S.xl, PC_M6_F2);
                if (S.ext_ret == 1) {
                    S.seq_pos = sp_corr(a, S, S.A, S.C, pos);
                    SP_CHECK();
                    if (S.seq_pos != 0xffffffffu) S.n_out = 2;
                }
            }
        }
        if (S.n_out == 2) {
            sp_copy(S.res0, S.A.a0);
            sp_copy(S.res1, S.C.a0);
            sp_splicing(S.res0);
            sp_splicing(S.res1);
        } else if (S.n_out > 0) {
            sp_copy(S.res0, S.C.a0);
            sp_splicing(S.res0);
        }
        SP_FINISH();
    default:
        S.status = HSA_SP_LOOP;
        SP_FINISH();
    }
}

__device__ __forceinline__ int sp_log2(uint32_t v)   // bwtgap.c:107-116
{
    int c = 0;
    if (v & 0xffff0000u) { v >>= 16; c |= 16; }
    if (v & 0xff00) { v >>= 8; c |= 8; }
    if (v & 0xf0) { v >>= 4; c |= 4; }
    if (v & 0xc) { v >>= 2; c |= 2; }
    if (v & 0x2) c |= 1;
    return c;
}

#ifdef HSA_SP_DIAG
__device__ unsigned long long g_spd[8];
#endif
__global__ void __launch_bounds__(SP_NT, 4) k_splice(SpArgs a)
{
    extern __shared__ uint32_t s_hn[];                 // per bucket: head | count << 16, lane-interleaved
    __shared__ uint8_t s_bmap[HSA_SP_MAX_STACKS];
    for (uint32_t i = threadIdx.x; i < HSA_SP_MAX_STACKS; i += SP_NT) s_bmap[i] = a.bmap[i];
    __syncthreads();
    const uint32_t lane = blockIdx.x * SP_NT + threadIdx.x;
    SpLane &S = a.lanes[lane];
    uint32_t *const lb = a.lbuf + (size_t)lane * a.lbuf_words;
    uint4 *const P = a.pool + (size_t)lane * a.cap * 2;
    uint32_t *const hn = s_hn + threadIdx.x;
    const int nst = (int)a.nb;                          // dense buckets
    const hsa_regime_t &R = a.rg;

    // ---- the extension in flight (bwt_backtracing_search, bwtgap.c:346-511; k_extend)
    bool x_on = false, x_pend = false;
    int x_dir = 0, x_len = 0, x_start = 0, x_end = 0, x_mp0 = 0, x_mp = 0, x_best = 0, x_nent = 0, x_pscore = 0;
    int x_err = 0, x_ret = 0, x_mode = 0, x_md = 0, x_L = 0, x_bscore = 0;
    uint32_t x_top = 0, x_freel = SP_NIL;
    uint4 x_pe0 = make_uint4(0, 0, 0, 0), x_pe1 = make_uint4(0, 0, 0, 0);
    uint32_t *x_aln = nullptr;           // the hit being extended: A.a0 (foreward) or C.a0 (backward), in place
    const uint8_t *x_seq = nullptr;
    const int32_t *x_w = nullptr, *x_w6 = nullptr;
    unsigned long long n_pops = 0, n_ext = 0, n_sa = 0;

    auto seq_at = [&](int p) -> uint32_t {
        if (p < 0 || p >= x_L) { x_err = HSA_SP_WIN; return 4u; }
        return x_seq[p];
    };
    auto bid_at = [&](int p) -> int {
        if (p < 0 || p > x_L) { x_err = HSA_SP_WIN; return 0; }
        if (x_w6 && p <= 12) return x_w6[2 * p + 1];
        return x_w[2 * p + 1];
    };
    auto flush = [&]() {                               // the pending entry into its bucket
        x_pend = false;
        uint32_t slot;
        if (x_freel != SP_NIL) { slot = x_freel; x_freel = P[(size_t)slot * 2 + 1].z; }
        else if (x_top < a.cap) slot = x_top++;
        else { x_err = HSA_SP_CAP; return; }
        const uint32_t v = hn[(uint32_t)x_pscore * SP_NT];
        x_pe1.z = (v >> 16) ? (v & 0xFFFFu) : SP_NIL;
        P[(size_t)slot * 2] = x_pe0;
        P[(size_t)slot * 2 + 1] = x_pe1;
        hn[(uint32_t)x_pscore * SP_NT] = slot | ((v >> 16) + 1u) << 16;
        if (x_best > x_pscore) x_best = x_pscore;
    };
    auto push = [&](int i, uint32_t k, uint32_t l, uint32_t rk, uint32_t rl, int mm, int go, int ge, int st) {
        const int score = mm * R.s_mm + go * R.s_gapo + ge * R.s_gape;      // gap_push (bwtgap.c:46-75)
        if (score < 0 || score >= R.n_stacks) { x_err = HSA_SP_SCORE; return; }
        const uint32_t bk = s_bmap[score];
        if (bk == 0xffu) { x_err = HSA_SP_SCORE; return; }
        if (x_pend) flush();
        x_pe0 = make_uint4(k, l, rk, rl);
        x_pe1 = make_uint4((uint32_t)score << 21 | (uint32_t)i,
                           (uint32_t)(mm & 255) | (uint32_t)(go & 255) << 8 | (uint32_t)(ge & 255) << 16 |
                               (uint32_t)(st & 3) << 24,
                           0u, 0u);
        x_pscore = (int)bk;                             // the bucket (score order)
        x_pend = true;
        ++x_nent;
    };
    auto step_all = [&](int backward, uint32_t k, uint32_t l, uint32_t rk, uint32_t rl, uint32_t ok[4], uint32_t ol[4],
                        uint32_t ork[4], uint32_t orl[4]) {
        uint32_t oL[4], oR[4], oC[4];
        const uint32_t p1 = backward ? k : rk, p2 = (backward ? l : rl) + 1u, lim = (backward ? a.T : a.rT) + 1u;
        if (p1 > lim || p2 > lim || p2 == 0u) { x_err = HSA_SP_RANK; return; }
        hsa_occ_pair(backward ? a.fwd : a.rev, p1, p2, oL, oR);
        oC[3] = 0;
        for (int c = 2; c >= 0; --c) oC[c] = oC[c + 1] + oR[c + 1] - oL[c + 1];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (backward) {
                ok[c] = a.C[c] + oL[c] + 1u;
                ol[c] = a.C[c] + oR[c];
                orl[c] = rl - oC[c];
                ork[c] = orl[c] - (ol[c] - ok[c]);
            } else {
                ork[c] = a.C[c] + oL[c] + 1u;
                orl[c] = a.C[c] + oR[c];
                ol[c] = l - oC[c];
                ok[c] = ol[c] - (orl[c] - ork[c]);
            }
        }
    };
    auto pk4 = [](const uint32_t v[4], uint32_t c) { return hsa_sel4<uint32_t>(c, v[0], v[1], v[2], v[3]); };
    // the extension S asks for (bwt_extend_foreward on A / bwt_extend_backward on C,
    // bwtgap.c:640-663): a fresh stack holding the hit
    auto ext_start = [&]() {
        const int rr = S.read;
        x_dir = S.xdir;
        x_len = S.xl;
        x_aln = x_dir ? S.C.a0 : S.A.a0;
        x_start = (int)x_aln[6];
        x_end = (int)x_aln[7];
        x_mp0 = x_mp = S.max_pos;
        x_mode = (R.mode & ~MODE_GAPE) | (S.gape ? MODE_GAPE : 0);
        x_md = a.pf.amd[rr];
        x_bscore = (x_md + 1) * R.s_mm + (R.max_gapo + 1) * R.s_gapo + (R.max_gape + 1) * R.s_gape;
        x_L = S.L;
        const int s = S.strand;
        x_seq = a.pf.scodes + (size_t)(2 * rr + s) * a.pf.sc;
        x_w = a.pf.rows + 2 * ((size_t)rr * 6u + (x_dir ? 0u : 4u) + (uint32_t)s) * a.pf.rs;   // width_back W1 / width_fore W0
        x_w6 = (x_dir && S.anchor6) ? a.pf.cw + 2 * (8 * (size_t)rr + 6 + s) * a.pf.cws : nullptr;
        for (int b = 0; b < nst; ++b) hn[(uint32_t)b * SP_NT] = 0;
        x_best = nst; x_nent = 0; x_top = 0; x_freel = SP_NIL; x_pend = false; x_err = 0; x_ret = 0;
        if (x_len < 0 && (x_mode & MODE_NONSTOP)) x_err = HSA_SP_WIN;    // a negative length read as 0xffff
        else
            push(x_len, x_aln[1], x_aln[2], x_aln[3], x_aln[4], (int)(x_aln[0] & 0xFFFFu), (int)((x_aln[0] >> 16) & 0xFFu),
                 (int)(x_aln[0] >> 24), ST_M);                                        // bwtgap.c:644 / :658
        x_on = true;
        ++n_ext;
    };
    auto ext_end = [&]() {
        x_on = false;
        if (!x_err && x_ret != 1) x_ret = x_mp != x_mp0 ? 2 : -1;
    };
    // one gap_pop and its expansion (bwtgap.c:371-504)
    auto ext_pop = [&]() {
        if (x_nent == 0 || x_err || x_nent > R.max_entries) { ext_end(); return; }
        ++n_pops;
        uint4 e0, e1;
        if (x_pend && x_pscore <= x_best) {
            e0 = x_pe0; e1 = x_pe1;
            x_pend = false;
            --x_nent;
        } else {
            if (x_pend) { flush(); if (x_err) { ext_end(); return; } }
            const uint32_t v = hn[(uint32_t)x_best * SP_NT];
            const uint32_t slot = v & 0xFFFFu, nb = (v >> 16) - 1u;
            e0 = P[(size_t)slot * 2]; e1 = P[(size_t)slot * 2 + 1];
            hn[(uint32_t)x_best * SP_NT] = (e1.z & 0xFFFFu) | nb << 16;
            --x_nent;
            P[(size_t)slot * 2 + 1].z = x_freel;
            x_freel = slot;
            if (nb == 0 && x_nent > 0) {
                int b = x_best + 1;
                while (b < nst && (hn[(uint32_t)b * SP_NT] >> 16) == 0) ++b;
                x_best = b;
            } else if (nb == 0) {
                x_best = nst;
            }
        }
        uint32_t k = e0.x, l = e0.y, rk = e0.z, rl = e0.w;
        const uint32_t info = e1.x;
        const int e_mm = (int)(e1.y & 255u), e_go = (int)((e1.y >> 8) & 255u), e_ge = (int)((e1.y >> 16) & 255u);
        const int e_st = (int)((e1.y >> 24) & 3u);
        int i = (int)(info & 0xffffu);
        if (!(x_mode & MODE_NONSTOP) && (int)(info >> 21) > x_bscore + R.s_mm) { ext_end(); return; }
        int m = x_md - (e_mm + e_go);
        if (x_mode & MODE_GAPE) m -= e_ge;
        const int len = x_len, bw = x_dir, start = x_start, end = x_end;
        if (m <= 0 || i == 0) {
            if (m == 0 && i != 0) {
                // bwt_extend_exact (2BWT-Interface.c:394-439)
                uint32_t xk = k, xl = l, xrk = rk, xrl = rl;
                if (bw == 1) {
                    const int s0 = start - len - 1;
                    while (i != 0 && !x_err) {
                        const uint32_t c = seq_at(s0 + i);
                        if (c > 3) break;
                        uint32_t ok[4], ol[4], ork[4], orl[4];
                        step_all(1, xk, xl, xrk, xrl, ok, ol, ork, orl);
                        xk = pk4(ok, c); xl = pk4(ol, c); xrk = pk4(ork, c); xrl = pk4(orl, c);
                        if (xk > xl) break;
                        k = xk; l = xl; rk = xrk; rl = xrl;
                        --i;
                    }
                } else {
                    const int rp = end + len - i + 1;          // start + leav - leav: fixed (:424)
                    while (!x_err) {
                        const uint32_t c = seq_at(rp);
                        if (c > 3) break;
                        uint32_t ok[4], ol[4], ork[4], orl[4];
                        step_all(0, xk, xl, xrk, xrl, ok, ol, ork, orl);
                        xk = pk4(ok, c); xl = pk4(ol, c); xrk = pk4(ork, c); xrl = pk4(orl, c);
                        if (xk > xl) break;
                        k = xk; l = xl; rk = xrk; rl = xrl;
                    }
                }
                if (x_err) { ext_end(); return; }
            }
            if (bw == 1 && x_mp >= start + i - len && (int)x_aln[6] > start + i - len) {
                x_aln[6] = (uint32_t)(start + i - len);
                x_mp = (int)x_aln[6];
            } else if (bw == 0 && x_mp <= end + len - i && (int)x_aln[7] < end + len - i) {
                x_aln[7] = (uint32_t)(end + len - i);
                x_mp = (int)x_aln[7];
            } else {
                return;
            }
            x_aln[1] = k; x_aln[2] = l; x_aln[3] = rk; x_aln[4] = rl;
            x_aln[5] = (x_aln[5] & 0xC0000000u) | 4u;                 // BWA_TYPE_SPLICING, strand kept
            x_aln[0] = (uint32_t)e_mm | (uint32_t)e_go << 16 | (uint32_t)e_ge << 24;
            x_aln[8] = info >> 21;
            if (i == 0) { x_ret = 1; ext_end(); }
            return;
        }
        --i;
        const int real_pos = bw == 1 ? start - len + i : len + end - i;
        uint32_t ok[4], ol[4], ork[4], orl[4];
        step_all(bw, k, l, rk, rl, ok, ol, ork, orl);
        if (x_err) { ext_end(); return; }
        const uint32_t occ = l - k + 1u;
        int allow_diff = 1;
        if (bw == 1 && x_mp < real_pos) {
            const int d = bid_at(real_pos) - bid_at(x_mp);
            if (d > m || (d == m && bid_at(x_mp) != bid_at(x_mp + 1))) allow_diff = 0;
        }
        if (bw == 0 && x_mp > real_pos) {
            const int d = bid_at(real_pos) - bid_at(x_mp);
            if (d > m || (d == m && bid_at(x_mp) != bid_at(x_mp - 1))) allow_diff = 0;
        }
        const int tmp = (x_mode & MODE_LOGGAP) ? sp_log2((uint32_t)(e_ge + e_go)) / 2 + 1 : e_go + e_ge;
        if (allow_diff && i >= R.indel_end_skip + tmp && len - i >= R.indel_end_skip + tmp) {
            if (e_st == ST_M) {
                if (e_go < R.max_gapo) {
                    push(i, k, l, rk, rl, e_mm, e_go + 1, e_ge, ST_I);
                    for (int j = 0; j != 4; ++j)
                        if ((bw == 1 && ok[j] <= ol[j]) || (bw == 0 && ork[j] <= orl[j]))
                            push(i + 1, ok[j], ol[j], ork[j], orl[j], e_mm, e_go + 1, e_ge, ST_D);
                }
            } else if (e_st == ST_I) {
                if (e_ge < R.max_gape) push(i, k, l, rk, rl, e_mm, e_go, e_ge + 1, ST_I);
            } else if (e_st == ST_D) {
                if (e_ge < R.max_gape && (e_ge + e_go < x_md || occ < (uint32_t)R.max_del_occ))
                    for (int j = 0; j != 4; ++j)
                        if (ok[j] <= ol[j]) push(i + 1, ok[j], ol[j], ork[j], orl[j], e_mm, e_go, e_ge + 1, ST_D);
            }
        }
        if (allow_diff == 1) {
            const uint32_t sc = seq_at(real_pos);
            for (int j = 1; j <= 4; ++j) {
                const uint32_t c = (sc + (uint32_t)j) & 3u;
                const int is_mm = (j != 4 || sc > 3) ? 1 : 0;
                if ((bw == 1 && pk4(ok, c) <= pk4(ol, c)) || (bw == 0 && pk4(ork, c) <= pk4(orl, c)))
                    push(i, pk4(ok, c), pk4(ol, c), pk4(ork, c), pk4(orl, c), e_mm + is_mm, e_go, e_ge, ST_M);
            }
        }
        if (x_err) ext_end();
    };

#ifdef HSA_SP_DIAG
    // diagnostic builds: wave time in the control and extension phases, lanes active in each
    uint64_t dg_ctrl = 0, dg_ext = 0, dg_all = __builtin_amdgcn_s_memtime();
    uint64_t dg_lctrl = 0, dg_lext = 0, dg_nctrl = 0, dg_next = 0;
#endif
    // ---- the lane's reads, one after another, from the batch's queue
    S.read = -1;
    S.n_ext = 0;
    S.n_sa = 0;
    bool done = false;
    int cur = -1;
    const unsigned long long n_reads = a.pf.d_n ? *a.pf.d_n : a.pf.n;
    for (;;) {
        if (!done && cur < 0 && !x_on) {
            const unsigned long long q = atomicAdd(a.next, 1ull);
            if (q >= n_reads) done = true;
            else { sp_init(a, S, (int)q); cur = (int)q; }
        }
        if (!__any(!done)) break;                       // every lane of the wave: queue empty, reads done
#ifdef HSA_SP_DIAG
        const uint64_t dg_t1 = __builtin_amdgcn_s_memtime();
        const uint64_t dg_bc = __ballot(!done && !x_on && cur >= 0);
#endif
        if (!done && !x_on && cur >= 0) {
            int c;
            do { c = sp_ctrl(a, S, lb); } while (c == SP_AGAIN);
            if (c == SP_EXT) ext_start();
            else cur = -1;
        }
#ifdef HSA_SP_DIAG
        const uint64_t dg_t2 = __builtin_amdgcn_s_memtime();
        const uint64_t dg_be = __ballot(x_on);
        if (dg_bc) { dg_ctrl += dg_t2 - dg_t1; dg_lctrl += (uint64_t)__popcll(dg_bc); ++dg_nctrl; }
#endif
        if (x_on) {                                     // one place for every lane's extension
            for (int q = 0; q < HSA_SP_BUDGET && x_on; ++q) ext_pop();
            if (!x_on) {
                if (x_err) {
                    S.status = x_err;
                    sp_finish(a, S);
                    cur = -1;
                } else {
                    S.max_pos = x_mp;
                    S.ext_ret = x_ret;
                }
            }
        }
#ifdef HSA_SP_DIAG
        if (dg_be) { dg_ext += __builtin_amdgcn_s_memtime() - dg_t2; dg_lext += (uint64_t)__popcll(dg_be); ++dg_next; }
#endif
    }
#ifdef HSA_SP_DIAG
    if ((threadIdx.x & 63u) == 0) {
        atomicAdd(&g_spd[0], dg_ctrl); atomicAdd(&g_spd[1], dg_ext);
        atomicAdd(&g_spd[2], __builtin_amdgcn_s_memtime() - dg_all);
        atomicAdd(&g_spd[3], dg_lctrl); atomicAdd(&g_spd[4], dg_nctrl);
        atomicAdd(&g_spd[5], dg_lext); atomicAdd(&g_spd[6], dg_next);
        __threadfence();
        if (atomicAdd(&g_spd[7], 1ull) + 1ull == (unsigned long long)gridDim.x * (SP_NT / 64)) {
            printf("[sp_diag] waves %llu: wave cycles control %llu ext %llu total %llu; control passes %llu (lanes %.1f per "
                   "pass), extension passes %llu (lanes %.1f per pass)\n", g_spd[7], g_spd[0], g_spd[1], g_spd[2], g_spd[4],
                   (double)g_spd[3] / (double)(g_spd[4] ? g_spd[4] : 1), g_spd[6],
                   (double)g_spd[5] / (double)(g_spd[6] ? g_spd[6] : 1));
            for (int i = 0; i < 8; ++i) g_spd[i] = 0;
        }
    }
#endif
    n_sa = S.n_sa;
    atomicAdd(a.ctr + 0, n_ext);
    atomicAdd(a.ctr + 1, n_pops);
    atomicAdd(a.ctr + 2, n_sa);
}

extern "C" int hsa_index_set_text(hsa_index_t *ix, const uint32_t *packed, uint64_t n_words, uint32_t dna_len)
{
    if (!packed || n_words == 0 || (uint64_t)dna_len > n_words * 16) {
        hsa_set_error("hsa_index_set_text: bad arguments");
        return HSA_E_ARG;
    }
    if (int rc0 = hsa_need32(ix)) return rc0;
    if (int rc0 = hsa_need_unshared(ix, "hsa_index_set_text")) return rc0;
    HSA_HIP(hipSetDevice(ix->device));
    (void)hipFree(ix->d_text);
    ix->d_text = nullptr;
    if (hipMalloc(&ix->d_text, n_words * 4) != hipSuccess) {
        (void)hipGetLastError();
        ix->d_text = nullptr;
        hsa_set_error("hsa_index_set_text: hipMalloc of %llu words failed", (unsigned long long)n_words);
        return HSA_E_MEM;
    }
    HSA_HIP(hipMemcpy(ix->d_text, packed, n_words * 4, hipMemcpyHostToDevice));
    ix->text_words = n_words;
    ix->dna_len = dna_len;
    return 0;
}

int hsa_splice_device_launch(hsa_index *ix, const PfDev &pd, const hsa_regime_t &rg, uint32_t *d_res,
                             unsigned long long *d_ctr, hipStream_t st)
{
    if (!ix->d_sa || !ix->d_text) {
        hsa_set_error("splice kernel: %s not attached", !ix->d_sa ? "the suffix array (hsa_index_set_sa)"
                                                                   : "the packed text (hsa_index_set_text)");
        return HSA_E_ARG;
    }
    if (rg.n_stacks < 1 || rg.n_stacks > HSA_SP_MAX_STACKS) {
        hsa_set_error("splice kernel: %d score buckets (at most %d)", rg.n_stacks, HSA_SP_MAX_STACKS);
        return HSA_E_ARG;
    }
    if (pd.n == 0) return 0;
    // The buckets: the scores an extension can reach, in score order.  Its entries'
    // counts: n_mm <= max(max_diff, max_seed_diff) (a seed's hit, or a child of an entry
    // with a difference left, bwtgap.c:389, :493-502), n_gapo <= max_gapo, n_gape <=
    // max_gape (:456, :472, :476; the anchors' hits have the same bounds).  A push outside
    // them is handed back (HSA_SP_SCORE), so the map never changes an answer.
    uint8_t bmap[HSA_SP_MAX_STACKS];
    memset(bmap, 0xff, sizeof bmap);
    const int mmx = rg.max_diff > rg.max_seed_diff ? rg.max_diff : rg.max_seed_diff;
    for (int mm = 0; mm <= mmx; ++mm)
        for (int go = 0; go <= rg.max_gapo; ++go)
            for (int ge = 0; ge <= rg.max_gape; ++ge) {
                const int sc = mm * rg.s_mm + go * rg.s_gapo + ge * rg.s_gape;
                if (sc >= 0 && sc < rg.n_stacks) bmap[sc] = 0;
            }
    uint32_t nb = 0;
    for (int sc = 0; sc < rg.n_stacks; ++sc)
        if (bmap[sc] == 0) bmap[sc] = (uint8_t)nb++;
    if (nb == 0) nb = 1;
    // workgroups per CU by the bucket table's LDS (160 KB per CU, 16 waves)
    const size_t lds = (size_t)nb * SP_NT * 4;
    int wpc = (int)((160u << 10) / (lds + HSA_SP_MAX_STACKS));
    wpc = wpc > 16 ? 16 : wpc < 1 ? 1 : wpc;
    const size_t resident = (size_t)(ix->n_cu > 0 ? ix->n_cu : 256) * (size_t)wpc * SP_NT;
    const size_t want = ((size_t)pd.n + SP_NT - 1) / SP_NT * SP_NT;
    const size_t lanes = want < resident ? want : resident;
    static const int cap_env = getenv("HSA_SPLICE_CAP") ? atoi(getenv("HSA_SPLICE_CAP")) : 0;
    const uint32_t cap = cap_env > 0 && cap_env <= 65535 ? (uint32_t)cap_env : 1024u;
    SpArgs A;
    memset(&A, 0, sizeof A);
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T; A.rT = ix->rT;
    memcpy(A.C, ix->C, sizeof A.C);
    A.sav = hsa_sa_view(ix);
    A.text = ix->d_text;
    A.text_chars = ix->text_words * 16;
    A.dna_len = ix->dna_len;
    A.pf = pd;
    A.rg = rg;
    A.nb = nb;
    memcpy(A.bmap, bmap, sizeof bmap);
    A.cap = cap;
    A.site_cap = 3 * pd.max_len + 8;
    A.ref_cap = pd.max_len + 8;
    A.lbuf_words = 3 * SP_POS_MAX + A.site_cap + (A.ref_cap + 3) / 4;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t b_pool = al(lanes * cap * 32), b_lanes = al(lanes * sizeof(SpLane)),
                 b_lbuf = al(lanes * A.lbuf_words * 4);
    int rc;
    if ((rc = hsa_grow(&ix->d_sp, &ix->d_sp_cap, b_pool + b_lanes + b_lbuf + 256))) return rc;
    char *d = (char *)ix->d_sp;
    A.pool = (uint4 *)d;
    A.lanes = (SpLane *)(d + b_pool);
    A.lbuf = (uint32_t *)(d + b_pool + b_lanes);
    A.next = (unsigned long long *)(d + b_pool + b_lanes + b_lbuf);
    A.ctr = d_ctr;
    A.res = d_res;
    HSA_HIP(hipMemsetAsync(A.next, 0, 8, st));
    HSA_HIP(hipMemsetAsync(d_ctr, 0, 4 * 8, st));
    hipLaunchKernelGGL(k_splice, dim3((unsigned)(lanes / SP_NT)), dim3(SP_NT), lds, st, A);
    HSA_HIP(hipGetLastError());
    if (getenv("HSA_VERBOSE"))
        fprintf(stderr, "[hsa] splice kernel: %u reads on %zu lanes (%d workgroups of %d per CU, %u buckets, %u-entry "
                        "stacks)\n", pd.n, lanes, wpc, SP_NT, nb, cap);
    return 0;
}
