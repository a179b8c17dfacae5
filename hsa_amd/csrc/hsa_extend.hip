// hsa_extend.hip -- the splice path's seed extensions, batched.
//
// bwt_splice_match (bwtgap.c:748) grows a mapped seed across the rest of the read
// with bwt_extend_backward / bwt_extend_foreward (bwtgap.c:640-663): a fresh stack
// holding the seed's hit, then bwt_backtracing_search (bwtgap.c:346-511) -- a
// best-first search over the same bucketed LIFO as bwt_match_gap, extending the
// interval backward on the forward BWT (BWTAllSARangesBackward_Bidirection,
// 2BWT-Interface.c:235) or forward on the reverse BWT
// (BWTAllSARangesForward_Bidirection, :274), pruned by the width bids of the read,
// with an exact tail (bwt_extend_exact, :394-439) once no difference is left.  It
// rewrites the hit (start or end, interval, counts, score, type) whenever it reaches
// further toward max_pos, and returns 1 (reached), 2 (moved) or -1.
//
// Here one lane per call.  The calls of one batch come from many reads (the drop-in
// runs the splice path of every fallback read of a batch as coroutines and hands each
// round of their extension calls to one launch, bwtext_gpu.c); each lane owns a stack
// in HBM: bucket counts and heads (one per score, as gap_stack_t) and a pool of
// 32-byte entries linked per bucket, popped slots reused through a free list.  A call
// reads its read only inside the window [lo, lo + n) its arguments determine
// (include/hsa_gpu.h); a read outside is reported, never performed.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsa_device.h"
#include "hsa_internal.h"

#define EXT_NT 64
#define EXT_LDS_NB 128     // buckets per lane kept in LDS: 64 lanes x 128 x 8 B = 64 KiB
#define EXT_NIL 0xFFFFFFFFu
#define MODE_GAPE 0x01
#define MODE_LOGGAP 0x04
#define MODE_NONSTOP 0x10
#define ST_M 0
#define ST_I 1
#define ST_D 2
// status codes of a call that could not be completed (ret = EXT_ERR - code)
#define EXT_ERR (-1000)
#define EXT_E_CAP 1        // stack capacity of this pass exceeded (re-run with a larger one)
#define EXT_E_SCORE 2      // an entry's score outside the stack's buckets (undefined in the reference)
#define EXT_E_RANK 3       // a rank position past the text (undefined in the reference)
#define EXT_E_WIN 4        // a read position outside the call's window
#define EXT_CONT (-999)    // sliced mode: not finished, state saved in its slot
#define EXT_STATE_U4 6     // saved state of a sliced call, in uint4

struct ExtArgs {
    RankDir fwd, rev;
    uint32_t T, rT;
    uint32_t C[4];
    const hsa_regime_t *regimes;
    const hsa_ext_job_t *jobs;
    const int32_t *job_list;     // optional: the jobs of a re-run pass
    int n;
    const uint8_t *codes;
    const int32_t *bids;
    uint4 *pool;                 // per lane: cap entries x 2 uint4
    uint32_t *heads, *cnt;       // per lane: nb each
    uint32_t cap, nb;
    uint32_t lds;                // bucket heads and counts in LDS (nb <= EXT_LDS_NB), else in heads/cnt
    uint32_t lnb;                // buckets per lane in the LDS layout
    // sliced mode (hsa_extend_sliced): lane t works on persistent slot slots[t] (its stack
    // and the state below stay in HBM between launches), resumes it when resume[t], and
    // stops after `budget` pops with ret = EXT_CONT
    const int32_t *slots;
    const uint8_t *resume;
    uint32_t budget;
    uint4 *state;                // per slot: EXT_STATE_U4 uint4
    int32_t *ret, *mp_out;
    uint32_t *aln_out;           // 9 words per job
};

__device__ __forceinline__ int ext_log2(uint32_t v)   // bwtgap.c:107-116
{
    int c = 0;
    if (v & 0xffff0000u) { v >>= 16; c |= 16; }
    if (v & 0xff00) { v >>= 8; c |= 8; }
    if (v & 0xf0) { v >>= 4; c |= 4; }
    if (v & 0xc) { v >>= 2; c |= 2; }
    if (v & 0x2) c |= 1;
    return c;
}

template <typename V> __device__ __forceinline__ V pk4(const V v[4], uint32_t c)
{
    return hsa_sel4<V>(c, v[0], v[1], v[2], v[3]);     // select tree (hsa_device.h)
}

__global__ void __launch_bounds__(EXT_NT) k_extend(ExtArgs a)
{
    const int t = blockIdx.x * EXT_NT + threadIdx.x;
    if (t >= a.n) return;
    const int jb = a.job_list ? a.job_list[t] : t;
    const hsa_ext_job_t J = a.jobs[jb];
    const hsa_regime_t R = a.regimes[J.regime];
    const size_t sl = a.slots ? (size_t)a.slots[t] : (size_t)t;   // the lane's stack region
    const bool resume = a.resume && a.resume[t];
    uint4 *const P = a.pool + sl * a.cap * 2;
    // bucket heads and counts (gap_stack_t's per-score stacks): lane-interleaved in LDS,
    // or per lane in HBM when there are too many buckets
    extern __shared__ uint32_t s_hn[];
    uint32_t *const Hb = a.lds ? s_hn + threadIdx.x : a.heads + sl * a.nb;
    uint32_t *const Nb = a.lds ? s_hn + (size_t)a.lnb * EXT_NT + threadIdx.x : a.cnt + sl * a.nb;
    const uint32_t hs = a.lds ? EXT_NT : 1u;
#define H(b) Hb[(uint32_t)(b) * hs]
#define N(b) Nb[(uint32_t)(b) * hs]
    const int nst = R.n_stacks;
    // sliced mode keeps the slot's heads and counts in HBM between launches; with the
    // bookkeeping in LDS they are copied in on resume and out when the call pauses
    uint32_t *const gH = a.heads + sl * a.nb, *const gN = a.cnt + sl * a.nb;
    if (!resume) {
        for (int b = 0; b < nst; ++b) N(b) = 0;
    } else if (a.lds) {
        for (int b = 0; b < nst; ++b) { H(b) = gH[b]; N(b) = gN[b]; }
    }
    int best = nst, n_ent = 0, err = 0;
    uint32_t top = 0, freel = EXT_NIL;
    const int len = J.len, bw = J.dir;
    const int lo = J.lo, hi = J.lo + J.n;
    const uint8_t *const sq = a.codes + J.off;
    const int32_t *const bd = a.bids + J.off;
    auto seq_at = [&](int p) -> uint32_t {
        if (p < lo || p >= hi) { err = EXT_E_WIN; return 4u; }
        return sq[p - lo];
    };
    auto bid_at = [&](int p) -> int {
        if (p < lo || p >= hi) { err = EXT_E_WIN; return 0; }
        return bd[p - lo];
    };
    // The entry pushed last stays in registers ("pending") until the next push or pop:
    // the next pop takes it whenever its score is <= the lowest non-empty bucket (it is
    // the top of that bucket then, bwtgap.c:77-92), so a chain of expansions whose last
    // child (the match, pushed last, bwtgap.c:493-502) is always the best never touches
    // the stack in HBM.
    bool pend = false;
    uint4 pe0 = make_uint4(0, 0, 0, 0), pe1 = make_uint4(0, 0, 0, 0);
    int pscore = 0;
    auto flush = [&]() {                               // the pending entry into its bucket
        pend = false;
        uint32_t slot;
        if (freel != EXT_NIL) { slot = freel; freel = P[(size_t)slot * 2 + 1].z; }
        else if (top < a.cap) slot = top++;
        else { err = EXT_E_CAP; return; }
        pe1.z = N(pscore) ? H(pscore) : EXT_NIL;
        P[(size_t)slot * 2] = pe0;
        P[(size_t)slot * 2 + 1] = pe1;
        H(pscore) = slot;
        ++N(pscore);
        if (best > pscore) best = pscore;
    };
    // gap_push (bwtgap.c:46-75): info = score << 21 | i in 32 bits; last_diff_pos is
    // never read by the extension
    auto push = [&](int i, uint32_t k, uint32_t l, uint32_t rk, uint32_t rl, int mm, int go, int ge, int st) {
        const int score = mm * R.s_mm + go * R.s_gapo + ge * R.s_gape;
        if (score < 0 || score >= nst) { err = EXT_E_SCORE; return; }
        if (pend) flush();
        pe0 = make_uint4(k, l, rk, rl);
        pe1 = make_uint4((uint32_t)score << 21 | (uint32_t)i,
                         (uint32_t)(mm & 255) | (uint32_t)(go & 255) << 8 | (uint32_t)(ge & 255) << 16 |
                             (uint32_t)(st & 3) << 24,
                         0u, 0u);
        pscore = score;
        pend = true;
        ++n_ent;
    };
    // one bidirectional step, all four characters: backward on the forward BWT, or
    // forward on the reverse BWT with the forward C table
    auto step_all = [&](int backward, uint32_t k, uint32_t l, uint32_t rk, uint32_t rl, uint32_t ok[4], uint32_t ol[4],
                        uint32_t ork[4], uint32_t orl[4]) {
        uint32_t oL[4], oR[4], oC[4];
        const uint32_t p1 = backward ? k : rk, p2 = (backward ? l : rl) + 1u, lim = (backward ? a.T : a.rT) + 1u;
        if (p1 > lim || p2 > lim || p2 == 0u) { err = EXT_E_RANK; return; }
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

    uint32_t aln[9];
#pragma unroll
    for (int w = 0; w < 9; ++w) aln[w] = J.aln[w];
    const int best_score = (R.max_diff + 1) * R.s_mm + (R.max_gapo + 1) * R.s_gapo + (R.max_gape + 1) * R.s_gape;
    const int max_diff = R.max_diff;
    const int start = (int)aln[6], end = (int)aln[7];    // the call's hit as given: fixed (bwtgap.c:365)
    int max_pos = J.max_pos, ret = 0;
    uint4 *const S = a.state ? a.state + sl * EXT_STATE_U4 : nullptr;
    if (resume) {                                         // a sliced call's saved state
        const uint4 s0 = S[0], s1 = S[1];
        best = (int)s0.x; n_ent = (int)s0.y; top = s0.z; freel = s0.w;
        pend = s1.x != 0; pscore = (int)s1.y; max_pos = (int)s1.z;
        pe0 = S[2]; pe1 = S[3];
        const uint4 a0 = S[4], a1 = S[5];
        aln[0] = a0.x; aln[1] = a0.y; aln[2] = a0.z; aln[3] = a0.w;
        aln[4] = a1.x; aln[5] = a1.y; aln[6] = a1.z; aln[7] = a1.w; aln[8] = s1.w;
    } else {
        push(len, aln[1], aln[2], aln[3], aln[4], (int)(aln[0] & 0xFFFFu), (int)((aln[0] >> 16) & 0xFFu),
             (int)(aln[0] >> 24), ST_M);                                    // bwtgap.c:644 / :658
    }
    uint32_t pops = 0;
    bool cont = false;
    while (n_ent != 0 && !err) {
        if (a.budget && pops == a.budget) { cont = true; break; }
        ++pops;
        if (n_ent > R.max_entries) break;
        // gap_pop (bwtgap.c:77-92)
        uint4 e0, e1;
        if (pend && pscore <= best) {
            e0 = pe0; e1 = pe1;
            pend = false;
            --n_ent;
        } else {
            if (pend) { flush(); if (err) break; }
            const uint32_t slot = H(best);
            e0 = P[(size_t)slot * 2]; e1 = P[(size_t)slot * 2 + 1];
            H(best) = e1.z;
            --N(best);
            --n_ent;
            P[(size_t)slot * 2 + 1].z = freel;
            freel = slot;
            if (N(best) == 0 && n_ent > (pend ? 1 : 0)) {
                int b = best + 1;
                while (b < nst && N(b) == 0) ++b;
                best = b;
            } else if (N(best) == 0) {
                best = nst;
            }
        }
        uint32_t k = e0.x, l = e0.y, rk = e0.z, rl = e0.w;
        const uint32_t info = e1.x;
        const int e_mm = (int)(e1.y & 255u), e_go = (int)((e1.y >> 8) & 255u), e_ge = (int)((e1.y >> 16) & 255u);
        const int e_st = (int)((e1.y >> 24) & 3u);
        int i = (int)(info & 0xffffu);
        if (!(R.mode & MODE_NONSTOP) && (int)(info >> 21) > best_score + R.s_mm) break;
        int m = max_diff - (e_mm + e_go);
        if (R.mode & MODE_GAPE) m -= e_ge;
        if (m <= 0 || i == 0) {
            if (m == 0 && i != 0) {
                // bwt_extend_exact (2BWT-Interface.c:394-439)
                uint32_t xk = k, xl = l, xrk = rk, xrl = rl;
                if (bw == 1) {
                    const int s0 = start - len + i - 1 - i;
                    while (i != 0 && !err) {
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
                    while (!err) {
                        const uint32_t c = seq_at(rp);
                        if (c > 3) break;
                        uint32_t ok[4], ol[4], ork[4], orl[4];
                        step_all(0, xk, xl, xrk, xrl, ok, ol, ork, orl);
                        xk = pk4(ok, c); xl = pk4(ol, c); xrk = pk4(ork, c); xrl = pk4(orl, c);
                        if (xk > xl) break;
                        k = xk; l = xl; rk = xrk; rl = xrl;
                    }
                }
                if (err) break;
            }
            if (bw == 1 && max_pos >= start + i - len && (int)aln[6] > start + i - len) {
                aln[6] = (uint32_t)(start + i - len);
                max_pos = (int)aln[6];
            } else if (bw == 0 && max_pos <= end + len - i && (int)aln[7] < end + len - i) {
                aln[7] = (uint32_t)(end + len - i);
                max_pos = (int)aln[7];
            } else {
                continue;
            }
            aln[1] = k; aln[2] = l; aln[3] = rk; aln[4] = rl;
            aln[5] = (aln[5] & 0xC0000000u) | 4u;                  // BWA_TYPE_SPLICING, strand kept
            aln[0] = (uint32_t)e_mm | (uint32_t)e_go << 16 | (uint32_t)e_ge << 24;
            aln[8] = info >> 21;
            if (i == 0) { ret = 1; break; }
            continue;
        }
        --i;
        const int real_pos = bw == 1 ? start - len + i : len + end - i;
        uint32_t ok[4], ol[4], ork[4], orl[4];
        step_all(bw, k, l, rk, rl, ok, ol, ork, orl);
        if (err) break;
        const uint32_t occ = l - k + 1u;
        int allow_diff = 1;
        if (bw == 1 && max_pos < real_pos) {
            const int d = bid_at(real_pos) - bid_at(max_pos);
            if (d > m || (d == m && bid_at(max_pos) != bid_at(max_pos + 1))) allow_diff = 0;
        }
        if (bw == 0 && max_pos > real_pos) {
            const int d = bid_at(real_pos) - bid_at(max_pos);
            if (d > m || (d == m && bid_at(max_pos) != bid_at(max_pos - 1))) allow_diff = 0;
        }
        const int tmp = (R.mode & MODE_LOGGAP) ? ext_log2((uint32_t)(e_ge + e_go)) / 2 + 1 : e_go + e_ge;
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
                if (e_ge < R.max_gape && (e_ge + e_go < max_diff || occ < (uint32_t)R.max_del_occ))
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
    }
    if (err) ret = EXT_ERR - err;
    else if (cont) {
        ret = EXT_CONT;
        if (a.lds)
            for (int b = 0; b < nst; ++b) { gH[b] = H(b); gN[b] = N(b); }
        S[0] = make_uint4((uint32_t)best, (uint32_t)n_ent, top, freel);
        S[1] = make_uint4(pend ? 1u : 0u, (uint32_t)pscore, (uint32_t)max_pos, aln[8]);
        S[2] = pe0; S[3] = pe1;
        S[4] = make_uint4(aln[0], aln[1], aln[2], aln[3]);
        S[5] = make_uint4(aln[4], aln[5], aln[6], aln[7]);
    } else if (ret != 1) ret = max_pos != J.max_pos ? 2 : -1;
    a.ret[jb] = ret;
    a.mp_out[jb] = max_pos;
#pragma unroll
    for (int w = 0; w < 9; ++w) a.aln_out[(size_t)jb * 9 + w] = aln[w];
#undef H
#undef N
}

// Device scratch of one pass: lanes x (cap entries x 32 B + nb x 8 B).
static int ext_scratch(hsa_index_t *ix, size_t lanes, uint32_t cap, uint32_t nb, uint4 **pool, uint32_t **heads,
                       uint32_t **cnt)
{
    const size_t pb = lanes * cap * 32, hb = lanes * nb * 4;
    int rc = hsa_grow(&ix->d_ext, &ix->d_ext_cap, pb + 2 * hb + 256);
    if (rc) return rc;
    *pool = (uint4 *)ix->d_ext;
    *heads = (uint32_t *)((char *)ix->d_ext + pb);
    *cnt = (uint32_t *)((char *)ix->d_ext + pb + hb);
    return 0;
}

extern "C" int hsa_extend_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_ext_job_t *jobs,
                                int n, const uint8_t *codes, const int32_t *bids, size_t win_len, int32_t *ret,
                                int32_t *max_pos, uint32_t *aln_out)
{
    if (n < 0 || n_regimes < 1 || (n > 0 && (!jobs || !regimes || !ret || !max_pos || !aln_out))) {
        hsa_set_error("hsa_extend_batch: bad arguments");
        return HSA_E_ARG;
    }
    if (n == 0) return 0;
    if (int rc0 = hsa_need32(ix)) return rc0;
    uint32_t nb = 1;
    int max_entries = 0;
    for (int r = 0; r < n_regimes; ++r) {
        if (regimes[r].n_stacks < 1 || regimes[r].n_stacks > 4096) {
            hsa_set_error("hsa_extend_batch: regime %d: n_stacks %d outside 1..4096", r, regimes[r].n_stacks);
            return HSA_E_ARG;
        }
        nb = (uint32_t)regimes[r].n_stacks > nb ? (uint32_t)regimes[r].n_stacks : nb;
        max_entries = regimes[r].max_entries > max_entries ? regimes[r].max_entries : max_entries;
    }
    for (int j = 0; j < n; ++j) {
        const hsa_ext_job_t &J = jobs[j];
        if (J.regime < 0 || J.regime >= n_regimes || J.n < 0 || (J.n > 0 && J.off + (uint64_t)J.n > win_len) ||
            (J.dir != 0 && J.dir != 1)) {
            hsa_set_error("hsa_extend_batch: call %d: bad job (regime %d, window %d at %llu of %zu)", j, J.regime, J.n,
                          (unsigned long long)J.off, win_len);
            return HSA_E_ARG;
        }
    }
    HSA_HIP(hipSetDevice(ix->device));
    ix->staged_valid = 0;                      // d_in is reused below
    const size_t rb = (size_t)n_regimes * sizeof(hsa_regime_t), jbb = (size_t)n * sizeof(hsa_ext_job_t);
    const size_t o_jobs = (rb + 255) / 256 * 256, o_codes = o_jobs + (jbb + 255) / 256 * 256;
    const size_t o_bids = o_codes + (win_len + 255) / 256 * 256, o_list = o_bids + (win_len * 4 + 255) / 256 * 256;
    const size_t inb = o_list + (size_t)n * 4 + 256;
    const size_t o_mp = ((size_t)n * 4 + 255) / 256 * 256, o_aln = o_mp + ((size_t)n * 4 + 255) / 256 * 256;
    const size_t outb = o_aln + (size_t)n * 36 + 256;
    int rc;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, inb)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, outb))) return rc;
    char *din = (char *)ix->d_in, *dout = (char *)ix->d_out;
    HSA_HIP(hipMemcpyAsync(din, regimes, rb, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, jbb, hipMemcpyHostToDevice, ix->stream));
    if (win_len) {
        HSA_HIP(hipMemcpyAsync(din + o_codes, codes, win_len, hipMemcpyHostToDevice, ix->stream));
        HSA_HIP(hipMemcpyAsync(din + o_bids, bids, win_len * 4, hipMemcpyHostToDevice, ix->stream));
    }
    ExtArgs A;
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T; A.rT = ix->rT;
    memcpy(A.C, ix->C, sizeof A.C);
    A.regimes = (const hsa_regime_t *)din;
    A.jobs = (const hsa_ext_job_t *)(din + o_jobs);
    A.codes = (const uint8_t *)(din + o_codes);
    A.bids = (const int32_t *)(din + o_bids);
    A.ret = (int32_t *)dout;
    A.mp_out = (int32_t *)(dout + o_mp);
    A.aln_out = (uint32_t *)(dout + o_aln);
    A.nb = nb;
    A.slots = nullptr; A.resume = nullptr; A.budget = 0; A.state = nullptr;
    // capacity passes: every call with a small stack, then the calls that overflowed it
    // with larger ones, up to what the reference's max_entries bound allows (live entries
    // <= max_entries + 9: the check precedes the pop, bwtgap.c:374)
    const uint32_t caps[3] = {256u, 65536u, (uint32_t)max_entries + 16u};
    const size_t budget = (size_t)8 << 30;     // scratch bytes per launch
    int32_t *list = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int n_run = n;
    for (int j = 0; j < n; ++j) list[j] = j;
    for (int pass = 0; pass < 3 && n_run > 0; ++pass) {
        const uint32_t cap = caps[pass];
        const size_t per = (size_t)cap * 32 + (size_t)nb * 8;
        const size_t chunk = budget / per > 0 ? budget / per : 1;
        HSA_HIP(hipMemcpyAsync(din + o_list, list, (size_t)n_run * 4, hipMemcpyHostToDevice, ix->stream));
        for (size_t c0 = 0; c0 < (size_t)n_run; c0 += chunk) {
            const size_t m = (size_t)n_run - c0 < chunk ? (size_t)n_run - c0 : chunk;
            if ((rc = ext_scratch(ix, m, cap, nb, &A.pool, &A.heads, &A.cnt))) { free(list); return rc; }
            A.cap = cap;
            A.job_list = (const int32_t *)(din + o_list) + c0;
            A.n = (int)m;
            A.lds = nb <= EXT_LDS_NB;
            A.lnb = nb;
            const size_t shm = A.lds ? (size_t)nb * EXT_NT * 8 : 0;
            hipLaunchKernelGGL(k_extend, dim3((unsigned)((m + EXT_NT - 1) / EXT_NT)), dim3(EXT_NT), shm, ix->stream, A);
            HSA_HIP(hipGetLastError());
        }
        HSA_HIP(hipMemcpyAsync(ret, dout, (size_t)n * 4, hipMemcpyDeviceToHost, ix->stream));
        HSA_HIP(hipStreamSynchronize(ix->stream));
        int k = 0;
        for (int t = 0; t < n_run; ++t)
            if (ret[list[t]] == EXT_ERR - EXT_E_CAP) list[k++] = list[t];
        n_run = k;
    }
    free(list);
    HSA_HIP(hipMemcpyAsync(max_pos, dout + o_mp, (size_t)n * 4, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipMemcpyAsync(aln_out, dout + o_aln, (size_t)n * 36, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    for (int j = 0; j < n; ++j) {
        if (ret[j] > EXT_ERR) continue;
        static const char *why[5] = {"", "stack capacity", "a score outside the stack's buckets",
                                     "a rank position past the text", "a read position outside the call's window"};
        const int e = EXT_ERR - ret[j];
        hsa_set_error("hsa_extend_batch: call %d needs %s (undefined in the reference or past max_entries)", j,
                      e >= 1 && e <= 4 ? why[e] : "?");
        return HSA_E_ARG;
    }
    return 0;
}

// ---------------------------------------------------------------- sliced mode
// The splice runner's calls (bwtext_gpu.c) come in rounds from coroutines that wait on
// them; one long search would hold every other read's next round.  So each launch runs
// every call in flight for at most `budget` pops: a call that finishes returns its
// result, one that does not keeps its stack and state in its slot (HBM, persistent
// across launches) and is resumed by the next launch, while the coroutines whose calls
// finished go on.  Slots hold EXT_SLICE_CAP entries and EXT_SLICE_NB buckets; a call
// that needs more reports EXT_E_CAP / EXT_E_SCORE here and is re-run by the caller
// through hsa_extend_batch.
#define EXT_SLICE_CAP 2048u
#define EXT_SLICE_NB ((uint32_t)HSA_EXT_SLICE_STACKS)

extern "C" int hsa_extend_sliced(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_ext_job_t *jobs,
                                 const int32_t *slots, const uint8_t *resume, int n, const uint8_t *codes,
                                 const int32_t *bids, size_t win_len, int n_slots, uint32_t budget, int32_t *ret,
                                 int32_t *max_pos, uint32_t *aln_out)
{
    if (n < 0 || n_regimes < 1 || n_slots < 1 || (n > 0 && (!jobs || !regimes || !slots || !resume || !ret ||
                                                           !max_pos || !aln_out))) {
        hsa_set_error("hsa_extend_sliced: bad arguments");
        return HSA_E_ARG;
    }
    if (n == 0) return 0;
    if (int rc0 = hsa_need32(ix)) return rc0;
    for (int r = 0; r < n_regimes; ++r)
        if (regimes[r].n_stacks < 1 || regimes[r].n_stacks > (int)EXT_SLICE_NB) {
            hsa_set_error("hsa_extend_sliced: regime %d: n_stacks %d outside 1..%u", r, regimes[r].n_stacks,
                          EXT_SLICE_NB);
            return HSA_E_ARG;
        }
    for (int j = 0; j < n; ++j) {
        const hsa_ext_job_t &J = jobs[j];
        if (J.regime < 0 || J.regime >= n_regimes || J.n < 0 || (J.n > 0 && J.off + (uint64_t)J.n > win_len) ||
            (J.dir != 0 && J.dir != 1) || slots[j] < 0 || slots[j] >= n_slots) {
            hsa_set_error("hsa_extend_sliced: call %d: bad job", j);
            return HSA_E_ARG;
        }
    }
    HSA_HIP(hipSetDevice(ix->device));
    ix->staged_valid = 0;
    // persistent slots: stacks, bucket heads and counts, state (grown, never shrunk:
    // contents survive between calls with the same n_slots)
    const size_t pb = (size_t)n_slots * EXT_SLICE_CAP * 32, hb = (size_t)n_slots * EXT_SLICE_NB * 4;
    const size_t sb = (size_t)n_slots * EXT_STATE_U4 * 16;
    int rc;
    if ((rc = hsa_grow(&ix->d_slices, &ix->d_slices_cap, pb + 2 * hb + sb + 256))) return rc;
    const size_t rb = (size_t)n_regimes * sizeof(hsa_regime_t), jbb = (size_t)n * sizeof(hsa_ext_job_t);
    const size_t o_jobs = (rb + 255) / 256 * 256, o_codes = o_jobs + (jbb + 255) / 256 * 256;
    const size_t o_bids = o_codes + (win_len + 255) / 256 * 256, o_slot = o_bids + (win_len * 4 + 255) / 256 * 256;
    const size_t o_res = o_slot + ((size_t)n * 4 + 255) / 256 * 256, inb = o_res + (size_t)n + 256;
    const size_t o_mp = ((size_t)n * 4 + 255) / 256 * 256, o_aln = o_mp + ((size_t)n * 4 + 255) / 256 * 256;
    const size_t outb = o_aln + (size_t)n * 36 + 256;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, inb)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, outb))) return rc;
    char *din = (char *)ix->d_in, *dout = (char *)ix->d_out;
    HSA_HIP(hipMemcpyAsync(din, regimes, rb, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, jbb, hipMemcpyHostToDevice, ix->stream));
    if (win_len) {
        HSA_HIP(hipMemcpyAsync(din + o_codes, codes, win_len, hipMemcpyHostToDevice, ix->stream));
        HSA_HIP(hipMemcpyAsync(din + o_bids, bids, win_len * 4, hipMemcpyHostToDevice, ix->stream));
    }
    HSA_HIP(hipMemcpyAsync(din + o_slot, slots, (size_t)n * 4, hipMemcpyHostToDevice, ix->stream));
    HSA_HIP(hipMemcpyAsync(din + o_res, resume, (size_t)n, hipMemcpyHostToDevice, ix->stream));
    ExtArgs A;
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T; A.rT = ix->rT;
    memcpy(A.C, ix->C, sizeof A.C);
    A.regimes = (const hsa_regime_t *)din;
    A.jobs = (const hsa_ext_job_t *)(din + o_jobs);
    A.job_list = nullptr;
    A.n = n;
    A.codes = (const uint8_t *)(din + o_codes);
    A.bids = (const int32_t *)(din + o_bids);
    A.pool = (uint4 *)ix->d_slices;
    A.heads = (uint32_t *)((char *)ix->d_slices + pb);
    A.cnt = (uint32_t *)((char *)ix->d_slices + pb + hb);
    A.state = (uint4 *)((char *)ix->d_slices + pb + 2 * hb);
    A.cap = EXT_SLICE_CAP;
    A.nb = EXT_SLICE_NB;
    int nbmax = 1;
    for (int r = 0; r < n_regimes; ++r) nbmax = regimes[r].n_stacks > nbmax ? regimes[r].n_stacks : nbmax;
    A.lds = nbmax <= (int)EXT_LDS_NB;
    A.lnb = (uint32_t)nbmax;
    A.slots = (const int32_t *)(din + o_slot);
    A.resume = (const uint8_t *)(din + o_res);
    A.budget = budget;
    A.ret = (int32_t *)dout;
    A.mp_out = (int32_t *)(dout + o_mp);
    A.aln_out = (uint32_t *)(dout + o_aln);
    static const bool trace = getenv("HSA_EXT_TRACE") != nullptr;
    if (trace) {
        HSA_HIP(hipStreamSynchronize(ix->stream));
        HSA_HIP(hipEventRecord(ix->ev0, ix->stream));
    }
    const size_t shm = A.lds ? (size_t)nbmax * EXT_NT * 8 : 0;
    hipLaunchKernelGGL(k_extend, dim3((unsigned)((n + EXT_NT - 1) / EXT_NT)), dim3(EXT_NT), shm, ix->stream, A);
    HSA_HIP(hipGetLastError());
    if (trace) {
        HSA_HIP(hipEventRecord(ix->ev1, ix->stream));
        HSA_HIP(hipEventSynchronize(ix->ev1));
        float ms = 0.f;
        HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
        fprintf(stderr, "[hsa_extend_sliced] %d calls, %zu window bytes, kernel %.3f ms\n", n, win_len, ms);
    }
    HSA_HIP(hipMemcpyAsync(ret, dout, (size_t)n * 4, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipMemcpyAsync(max_pos, dout + o_mp, (size_t)n * 4, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipMemcpyAsync(aln_out, dout + o_aln, (size_t)n * 36, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    return 0;
}
