// hsa_search.hip -- the bwa_cal_sa_reg_gap per-read loop as one persistent kernel.
//
// One lane owns one read at a time (reads are pulled from a global queue with a
// wave-aggregated atomic, so a lane that finishes a cheap read immediately takes
// the next one: work-stealing at read granularity).  Per read the lane runs the
// reference's sequence exactly (bwtaln.c:343-373):
//   for strand = rc, fwd:  bwt_cal_width(seed) ; bwt_cal_width(read) ; bwt_match_gap
//   first strand with hits wins; no hit on either -> HSA_F_FALLBACK (splice).
//
// Every loop iteration of the kernel performs at most ONE bidirectional rank step
// per lane (two Occ queries on one BWT, usually one 64-byte block), whatever the
// lane is doing -- width extension, exact tail (bwt_match_exact) or expansion --
// so all lanes issue their HBM loads together and the state machine in between
// is register work.  Control that needs no rank (pruned pops, hits) loops
// without touching the BWT.
//
// Stack (bwtgap.c:13-92): n_stacks score buckets, each a LIFO.  Here each
// bucket is a singly linked list through a per-lane pool in HBM (16-byte entry +
// 16-bit link), bucket heads live in LDS, a 128-bit mask in registers gives the
// lowest non-empty bucket (== gap_stack_t.best).  The child pushed LAST by an
// expansion is always the next pop (it is the top of the lowest bucket), so it
// is kept in registers and never written ("virtual top").
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsa_device.h"
#include "hsa_internal.h"

#define MODE_GAPE 0x01
#define MODE_LOGGAP 0x04
#define MODE_NONSTOP 0x10
#define ST_M 0
#define ST_I 1
#define ST_D 2
#define NIL16 0xFFFFu
#define BLOCK 256

enum : int { PH_IDLE = 0, PH_WIDTH, PH_POP, PH_EXACT, PH_EXPAND, PH_EXIT };

struct SearchArgs {
    RankDir fwd, rev;
    uint32_t T;
    uint32_t C[5];
    const hsa_regime_t *regimes;
    const hsa_job_t *jobs;
    const int32_t *job_list;       // optional indirection (re-runs); null = identity
    int n_jobs;
    const uint8_t *codes;
    int32_t *n_aln;
    uint32_t *flags;
    uint64_t *hit_off;
    uint32_t *hits;
    uint64_t hit_cap;
    unsigned long long *ctr;       // [0] queue head [1] hit alloc [2] rank queries [3] blocks [4] pops
    uint2 *width;                  // per lane wcap entries: back [0, maxl+1), seed [maxl+1, wcap)
    uint4 *pool;
    uint16_t *nxt;
    uint32_t *hbuf;
    uint32_t wcap, seed_base, pcap, hcap, nb;
};

// entry meta word: i:10 | state:2 | is_diff:1 | n_mm:7 | n_gapo:4 | n_gape:8
__device__ __forceinline__ uint32_t meta_pack(int i, int st, int isd, int mm, int go, int ge)
{
    return (uint32_t)i | (uint32_t)st << 10 | (uint32_t)isd << 12 | (uint32_t)mm << 13 | (uint32_t)go << 20 |
           (uint32_t)ge << 24;
}

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

__global__ void __launch_bounds__(BLOCK) k_search(SearchArgs a)
{
    extern __shared__ uint16_t s_heads[];   // [nb][BLOCK]
    const uint32_t tid = threadIdx.x;
    const size_t gid = (size_t)blockIdx.x * BLOCK + tid;
    const int lane = (int)(tid & 63);
    uint2 *const wb = a.width + gid * a.wcap;
    uint2 *const ws = wb + a.seed_base;
    uint4 *const pool = a.pool + gid * a.pcap;
    uint16_t *const nxt = a.nxt + gid * a.pcap;
    uint32_t *const hb = a.hbuf + gid * (size_t)a.hcap * 9;
#define HEAD(b) s_heads[(size_t)(b) * BLOCK + tid]

    // ---- per-read state
    int ph = PH_IDLE;
    int job = -1;
    uint64_t off = 0;
    int len = 0, strand = 1, has_seed = 0, seed_len = 0, opt_max_diff = 0;
    hsa_regime_t R;
    // width
    int wpos = 0, wlen = 0, wstart = 0, wseed = 0, wbid = 0;
    uint32_t wk = 0, wl = 0;
    // search
    int best_score = 0, best_diff = 0, max_diff = 0, best_cnt = 0, n_aln = 0, n_entries = 0;
    uint32_t pool_top = 0;
    uint64_t mask0 = 0, mask1 = 0;
    int has_vt = 0;
    uint4 vt = make_uint4(0, 0, 0, 0);
    int pend = 0, pend_score = 0;
    uint4 pendv = make_uint4(0, 0, 0, 0);
    // current entry
    uint32_t ek = 0, el = 0, erk = 0, erl = 0;
    int ei = 0, est = 0, eisd = 0, emm = 0, ego = 0, ege = 0, em = 0, em_seed = 0;
    // exact tail
    uint32_t xk = 0, xl = 0, xrk = 0, xrl = 0;
    int xj = 0;
    // statistics
    uint64_t st_q = 0, st_b = 0, st_p = 0;
    int overflow = 0;

    auto getc = [&](int p) -> uint32_t {
        uint32_t c = a.codes[off + (strand ? (uint64_t)(len - 1 - p) : (uint64_t)p)];
        return strand ? (c < 4 ? 3u - c : c) : c;
    };
    auto score_of = [&](int mm, int go, int ge) -> int { return mm * R.s_mm + go * R.s_gapo + ge * R.s_gape; };

    auto start_width = [&]() {
        wseed = has_seed;
        wstart = has_seed ? len - seed_len : 0;
        wlen = has_seed ? seed_len : len;
        wpos = 0; wk = 0; wl = a.T; wbid = 0;
        ph = PH_WIDTH;
    };
    auto flush = [&](uint4 v, int b) {
        if (pool_top >= a.pcap || (uint32_t)b >= a.nb) { overflow = 1; return; }
        const uint32_t slot = pool_top++;
        const bool nonempty = b < 64 ? ((mask0 >> b) & 1ull) : ((mask1 >> (b - 64)) & 1ull);
        pool[slot] = v;
        nxt[slot] = nonempty ? HEAD(b) : (uint16_t)NIL16;
        HEAD(b) = (uint16_t)slot;
        if (b < 64) mask0 |= 1ull << b; else mask1 |= 1ull << (b - 64);
    };
    auto push = [&](int i, uint32_t k, uint32_t l, uint32_t rk, int mm, int go, int ge, int st, int isd) {
        if (pend) flush(pendv, pend_score);
        pendv = make_uint4(k, l, rk, meta_pack(i, st, isd, mm, go, ge));
        pend_score = score_of(mm, go, ge);
        pend = 1;
        ++n_entries;
    };
    auto start_search = [&]() {
        best_score = score_of(opt_max_diff + 1, R.max_gapo + 1, R.max_gape + 1);
        best_diff = opt_max_diff + 1;
        max_diff = opt_max_diff;
        best_cnt = 0; n_aln = 0;
        mask0 = mask1 = 0; pool_top = 0; pend = 0;
        // root entry (bwtgap.c:142) as the virtual top
        vt = make_uint4(0, a.T, 0, meta_pack(len, ST_M, 0, 0, 0, 0));
        has_vt = 1;
        n_entries = 1;
        ph = PH_POP;
    };
    auto finish_job = [&](uint32_t fl, int na, uint64_t ho) {
        a.n_aln[job] = na;
        a.flags[job] = fl;
        a.hit_off[job] = ho;
        ph = PH_IDLE;
    };
    auto end_strand = [&]() {
        if (n_aln > 0) {
            const unsigned long long o = atomicAdd(&a.ctr[1], (unsigned long long)n_aln);
            if (o + (uint64_t)n_aln > a.hit_cap) { finish_job(HSA_F_OVERFLOW, 0, 0); return; }
            uint32_t *dst = a.hits + o * 9;
            for (int h = 0; h < n_aln; ++h) {
                const uint32_t *s = hb + h * 9;
                dst[h * 9 + 0] = s[0];
                dst[h * 9 + 1] = s[1];
                dst[h * 9 + 2] = s[2];
                dst[h * 9 + 3] = s[3];
                dst[h * 9 + 4] = s[4];
                dst[h * 9 + 5] = (uint32_t)strand << 30;
                dst[h * 9 + 6] = 0;
                dst[h * 9 + 7] = h == 0 ? (uint32_t)(len - 1) : 0u;   // bwtaln.c:371-372
                dst[h * 9 + 8] = s[8];
            }
            finish_job(0, n_aln, o);
        } else if (strand == 1) {
            strand = 0;
            start_width();
        } else {
            finish_job(HSA_F_FALLBACK, 0, 0);
        }
    };
    // hit handling (bwtgap.c:188-243); returns false when the search must stop
    auto on_hit = [&](uint32_t k, uint32_t l, uint32_t rk, uint32_t rl) -> bool {
        const int score = score_of(emm, ego, ege);
        if (n_aln == 0) {
            best_score = score;
            best_diff = emm + ego + ((R.mode & MODE_GAPE) ? ege : 0);
            if (!(R.mode & MODE_NONSTOP)) max_diff = (best_diff + 1 > opt_max_diff) ? opt_max_diff : best_diff + 1;
        }
        if (score == best_score) best_cnt = (int)((uint32_t)best_cnt + (l - k + 1u));
        else if (best_cnt > R.max_top2) return false;
        bool add = true;
        if (ego) {
            for (int j = 0; j < n_aln; ++j)
                if (hb[j * 9 + 1] == k && hb[j * 9 + 2] == l) { add = false; break; }
        }
        if (add) {
            if ((uint32_t)n_aln >= a.hcap) { overflow = 1; return false; }
            // gap_shadow (bwtgap.c:94-105) on width_back[0, last_diff_pos)
            const uint32_t x = l - k + 1u;
            const int ldp = eisd ? ei : 0;
            uint32_t jj = 0;
            for (int p = 0; p < ldp; ++p) {
                uint2 w = wb[p];
                if (w.x > x) { w.x -= x; wb[p] = w; }
                else if (w.x == x) { w.y = 1; w.x = a.T - (++jj); wb[p] = w; }
            }
            uint32_t *h = hb + n_aln * 9;
            h[0] = (uint32_t)emm | (uint32_t)ego << 16 | (uint32_t)ege << 24;
            h[1] = k; h[2] = l; h[3] = rk; h[4] = rl;
            h[8] = (uint32_t)score;
            ++n_aln;
        }
        return true;
    };

    // request for this iteration's rank step
    int req = 0, rdir = 0;
    uint32_t rp1 = 0, rp2 = 0;

    for (;;) {
        // ---------------- (A) read acquisition, wave aggregated
        {
            const bool need = (ph == PH_IDLE);
            const uint64_t m = __ballot(need);
            if (m) {
                const int leader = __ffsll((unsigned long long)m) - 1;
                unsigned long long base = 0;
                if (lane == leader) base = atomicAdd(&a.ctr[0], (unsigned long long)__popcll(m));
                base = __shfl(base, leader);
                if (need) {
                    const unsigned long long j = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
                    if (j < (unsigned long long)a.n_jobs) {
                        job = a.job_list ? a.job_list[j] : (int)j;
                        const hsa_job_t J = a.jobs[job];
                        off = J.off; len = (int)J.len; opt_max_diff = J.max_diff;
                        seed_len = J.seed_len;
                        R = a.regimes[J.regime];
                        has_seed = len > seed_len;
                        strand = 1;
                        overflow = 0;
                        start_width();
                    } else {
                        ph = PH_EXIT;
                    }
                }
            }
        }
        if (__all(ph == PH_EXIT)) break;

        // ---------------- (B) control until a rank step is needed
        req = 0;
        while (ph != PH_EXIT && ph != PH_IDLE && !req) {
            if (overflow) { finish_job(HSA_F_OVERFLOW, 0, 0); break; }
            if (ph == PH_WIDTH) {
                // bwt_cal_width type 1 (bwtaln.c:84-97)
                while (wpos < wlen) {
                    const uint32_t c = getc(wstart + wpos);
                    if (c < 4) break;
                    wk = 0; wl = a.T; ++wbid;                               // N: restart
                    (wseed ? ws : wb)[wpos] = make_uint2(wl - wk + 1u, (uint32_t)wbid);
                    ++wpos;
                }
                if (wpos < wlen) { req = 1; rdir = 1; rp1 = wk; rp2 = wl + 1u; break; }
                (wseed ? ws : wb)[wlen] = make_uint2(0u, (uint32_t)(++wbid));
                if (wseed) { wseed = 0; wstart = 0; wlen = len; wpos = 0; wk = 0; wl = a.T; wbid = 0; }
                else start_search();
                continue;
            }
            if (ph == PH_EXACT) {
                const uint32_t c = getc(xj);
                if (c > 3) { ph = PH_POP; continue; }                     // 2BWT-Interface.c:377
                req = 1; rdir = 0; rp1 = xk; rp2 = xl + 1u;
                break;
            }
            // PH_POP: bwtgap.c:144-186
            if (n_entries == 0 || n_entries > R.max_entries) { end_strand(); continue; }
            uint4 e;
            if (has_vt) {
                e = vt; has_vt = 0;
            } else {
                int b;
                if (mask0) b = __ffsll((unsigned long long)mask0) - 1;
                else b = 64 + __ffsll((unsigned long long)mask1) - 1;
                const uint32_t slot = HEAD(b);
                e = pool[slot];
                const uint16_t nx = nxt[slot];
                if (nx == NIL16) { if (b < 64) mask0 &= ~(1ull << b); else mask1 &= ~(1ull << (b - 64)); }
                else HEAD(b) = nx;
            }
            --n_entries;
            ++st_p;
            ek = e.x; el = e.y; erk = e.z; erl = erk + (el - ek);
            ei = (int)(e.w & 1023u); est = (int)((e.w >> 10) & 3u); eisd = (int)((e.w >> 12) & 1u);
            emm = (int)((e.w >> 13) & 127u); ego = (int)((e.w >> 20) & 15u); ege = (int)(e.w >> 24);
            if (!(R.mode & MODE_NONSTOP) && score_of(emm, ego, ege) > best_score + R.s_mm) { end_strand(); continue; }
            em = max_diff - (emm + ego);
            if (R.mode & MODE_GAPE) em -= ege;
            if (em < 0) continue;
            if (has_seed) {
                em_seed = R.max_seed_diff - (emm + ego);
                if (R.mode & MODE_GAPE) em_seed -= ege;
            }
            if (ei > 0 && em < (int)wb[ei - 1].y) continue;
            if (ei == 0) {
                if (!on_hit(ek, el, erk, erl) && !overflow) end_strand();
                continue;
            }
            if (em == 0 && (est == ST_M || (R.mode & MODE_GAPE) || ege == R.max_gape)) {
                xk = ek; xl = el; xrk = erk; xrl = erl; xj = ei - 1;
                ph = PH_EXACT;
                continue;
            }
            --ei;
            req = 1; rdir = 0; rp1 = ek; rp2 = el + 1u;
            ph = PH_EXPAND;
        }

        // ---------------- (C) the rank step
        uint32_t oa[4], ob[4];
        if (req) {
            st_b += hsa_occ_pair(rdir ? a.rev : a.fwd, rp1, rp2, oa, ob);
            st_q += 2;
        }

        // ---------------- (D) apply
        if (req && ph == PH_WIDTH) {
            const uint32_t c = getc(wstart + wpos);
            wk = a.C[c] + oa[c] + 1u;
            wl = a.C[c] + ob[c];
            if (wk > wl) { wk = 0; wl = a.T; ++wbid; }
            (wseed ? ws : wb)[wpos] = make_uint2(wl - wk + 1u, (uint32_t)wbid);
            ++wpos;
        } else if (req && ph == PH_EXACT) {
            // BWTSARangeBackward_Bidirection (2BWT-Interface.c:135-170), one character
            const uint32_t c = getc(xj);
            uint32_t oc = 0;
            for (uint32_t d = c + 1; d < 4; ++d) oc += ob[d] - oa[d];
            const uint32_t nk = a.C[c] + oa[c] + 1u, nl = a.C[c] + ob[c];
            const uint32_t nrl = xrl - oc;
            xk = nk; xl = nl; xrl = nrl; xrk = nrl - (nl - nk);
            if (xk > xl) {
                ph = PH_POP;                                             // no match: continue (bwtgap.c:185)
            } else if (--xj < 0) {
                // write-back guard of bwt_match_exact (2BWT-Interface.c:383-386)
                const uint32_t hk = ek ? xk : ek, hl = el ? xl : el, hrk = erk ? xrk : erk, hrl = erl ? xrl : erl;
                ph = PH_POP;
                if (!on_hit(hk, hl, hrk, hrl) && !overflow) end_strand();
            }
        } else if (req && ph == PH_EXPAND) {
            // children of the bidirectional step (2BWT-Interface.c:235-272)
            uint32_t sk[4], sl[4], srk[4], oc[4];
            oc[3] = 0;
            for (int c = 2; c >= 0; --c) oc[c] = oc[c + 1] + ob[c + 1] - oa[c + 1];
            for (int c = 0; c < 4; ++c) {
                sk[c] = a.C[c] + oa[c] + 1u;
                sl[c] = a.C[c] + ob[c];
                const uint32_t rl = erl - oc[c];
                srk[c] = rl - (sl[c] - sk[c]);
            }
            const int i = ei;
            const uint32_t occ = el - ek + 1u;
            int allow_diff = 1, allow_M = 1;
            if (i > 0) {
                const uint2 w1 = wb[i - 1], w0 = wb[i];
                if ((int)w1.y > em - 1) allow_diff = 0;
                else if ((int)w1.y == em - 1 && (int)w0.y == em - 1 && w1.x == w0.x) allow_M = 0;
                const int ii = i - (len - seed_len);
                if (has_seed && ii > 0) {
                    const uint2 s1 = ws[ii - 1], s0 = ws[ii];
                    if ((int)s1.y > em_seed - 1) allow_diff = 0;
                    else if ((int)s1.y == em_seed - 1 && (int)s0.y == em_seed - 1 && s1.x == s0.x) allow_M = 0;
                }
            }
            const int tmp = (R.mode & MODE_LOGGAP) ? int_log2((uint32_t)(ege + ego)) / 2 + 1 : ego + ege;
            if (allow_diff && i >= R.indel_end_skip + tmp && len - i >= R.indel_end_skip + tmp) {
                if (est == ST_M) {
                    if (ego < R.max_gapo) {
                        push(i, ek, el, erk, emm, ego + 1, ege, ST_I, 1);
                        for (int j = 0; j < 4; ++j)
                            if (sk[j] <= sl[j]) push(i + 1, sk[j], sl[j], srk[j], emm, ego + 1, ege, ST_D, 1);
                    }
                } else if (est == ST_I) {
                    if (ege < R.max_gape) push(i, ek, el, erk, emm, ego, ege + 1, ST_I, 1);
                } else if (est == ST_D) {
                    if (ege < R.max_gape && (ege + ego < max_diff || occ < (uint32_t)R.max_del_occ)) {
                        for (int j = 0; j < 4; ++j)
                            if (sk[j] <= sl[j]) push(i + 1, sk[j], sl[j], srk[j], emm, ego, ege + 1, ST_D, 1);
                    }
                }
            }
            const uint32_t sc = getc(i);
            if (allow_diff && allow_M) {
                for (int j = 1; j <= 4; ++j) {
                    const int c = (int)((sc + (uint32_t)j) & 3u);
                    const int is_mm = (j != 4 || sc > 3);
                    if (sk[c] <= sl[c]) push(i, sk[c], sl[c], srk[c], emm + is_mm, ego, ege, ST_M, is_mm);
                }
            } else if (sc < 4) {
                const int c = (int)sc;
                if (sk[c] <= sl[c]) push(i, sk[c], sl[c], srk[c], emm, ego, ege, ST_M, 0);
            }
            // the last child: next pop if no memory bucket is lower (virtual top)
            if (pend) {
                int low = 1 << 30;
                if (mask0) low = __ffsll((unsigned long long)mask0) - 1;
                else if (mask1) low = 64 + __ffsll((unsigned long long)mask1) - 1;
                if (pend_score <= low) { vt = pendv; has_vt = 1; }
                else flush(pendv, pend_score);
                pend = 0;
            }
            ph = PH_POP;
        }
    }

    // statistics
    atomicAdd(&a.ctr[2], (unsigned long long)st_q);
    atomicAdd(&a.ctr[3], (unsigned long long)st_b);
    atomicAdd(&a.ctr[4], (unsigned long long)st_p);
#undef HEAD
}

// ---------------------------------------------------------------- host side
static int check_regimes(const hsa_regime_t *rg, int n)
{
    for (int r = 0; r < n; ++r) {
        const hsa_regime_t &R = rg[r];
        if (R.s_mm < 0 || R.s_gapo < 0 || R.s_gape < 0) { hsa_set_error("negative penalty"); return HSA_E_ARG; }
        if (R.n_stacks <= 0 || R.n_stacks > 128) { hsa_set_error("n_stacks %d outside 1..128", R.n_stacks); return HSA_E_ARG; }
        if (R.max_gapo > 14 || R.max_gape > 254) { hsa_set_error("max_gapo/max_gape out of range"); return HSA_E_ARG; }
    }
    return 0;
}

struct LaunchPlan {
    size_t lanes, blocks;
    uint32_t wcap, seed_base, pcap, hcap, nb;
    size_t lds;
};

static int plan_launch(hsa_index *ix, int n_jobs, int max_len, int max_seed, int nb, bool big, LaunchPlan &P)
{
    P.nb = (uint32_t)nb;
    P.lds = (size_t)nb * BLOCK * sizeof(uint16_t);
    int per_cu = 0;
    HSA_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_search, BLOCK, P.lds));
    const int want = g_waves_per_cu / (BLOCK / 64);
    if (per_cu > want) per_cu = want > 0 ? want : 1;
    if (per_cu < 1) { hsa_set_error("search kernel does not fit (LDS %zu)", P.lds); return HSA_E_ARG; }
    size_t blocks = (size_t)ix->n_cu * per_cu;
    size_t need_blocks = ((size_t)n_jobs + BLOCK - 1) / BLOCK;
    if (big) {
        blocks = need_blocks < 4 ? need_blocks : 4;
    } else if (need_blocks < blocks) {
        blocks = need_blocks;
    }
    if (blocks < 1) blocks = 1;
    P.blocks = blocks;
    P.lanes = blocks * BLOCK;
    P.seed_base = (uint32_t)max_len + 1;
    P.wcap = P.seed_base + (uint32_t)max_seed + 1;
    P.pcap = big ? 65535u : (uint32_t)g_pool_entries;
    P.hcap = big ? 16384u : (uint32_t)g_hit_cap;
    return 0;
}

// Launch one search pass over jobs (or job_list subset) with device pointers.
static int launch_pass(hsa_index *ix, const LaunchPlan &P, SearchScratch &S, const hsa_regime_t *d_regimes,
                       const hsa_job_t *d_jobs, const int32_t *d_list, int n, const uint8_t *d_codes,
                       int32_t *d_n, uint32_t *d_fl, uint64_t *d_ho, uint32_t *d_hits, uint64_t hit_cap,
                       unsigned long long *d_ctr, hipStream_t st)
{
    int rc = hsa_scratch_reserve(S, P.lanes, P.wcap, P.pcap, P.hcap);
    if (rc) return rc;
    SearchArgs A;
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T;
    memcpy(A.C, ix->C, sizeof A.C);
    A.regimes = d_regimes; A.jobs = d_jobs; A.job_list = d_list; A.n_jobs = n; A.codes = d_codes;
    A.n_aln = d_n; A.flags = d_fl; A.hit_off = d_ho; A.hits = d_hits; A.hit_cap = hit_cap; A.ctr = d_ctr;
    A.width = S.width; A.pool = S.pool; A.nxt = S.nxt; A.hbuf = S.hbuf;
    A.wcap = (uint32_t)S.wcap; A.seed_base = P.seed_base; A.pcap = (uint32_t)S.pcap; A.hcap = (uint32_t)S.hcap;
    A.nb = P.nb;
    HSA_HIP(hipMemsetAsync(d_ctr, 0, 8 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_search, dim3((unsigned)P.blocks), dim3(BLOCK), P.lds, st, A);
    HSA_HIP(hipGetLastError());
    return 0;
}

static int jobs_limits(const hsa_job_t *jobs, int n, int &max_len, int &max_seed)
{
    max_len = 0; max_seed = 0;
    for (int j = 0; j < n; ++j) {
        if (jobs[j].len > 1023) { hsa_set_error("read %d longer than 1023", j); return HSA_E_ARG; }
        if (jobs[j].max_diff > 125 || jobs[j].max_diff < -1) { hsa_set_error("max_diff out of range"); return HSA_E_ARG; }
        if ((int)jobs[j].len > max_len) max_len = (int)jobs[j].len;
        if ((int)jobs[j].len > jobs[j].seed_len && jobs[j].seed_len > max_seed) max_seed = jobs[j].seed_len;
    }
    return 0;
}

extern "C" long hsa_search_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                                 int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                                 uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats)
{
    *hits_out = nullptr;
    if (n_regimes < 1 || n_regimes > 2) { hsa_set_error("1 or 2 regimes"); return HSA_E_ARG; }
    int rc = check_regimes(regimes, n_regimes);
    if (rc) return rc;
    int max_len, max_seed;
    if ((rc = jobs_limits(jobs, n_jobs, max_len, max_seed))) return rc;
    int nb = 0;
    for (int r = 0; r < n_regimes; ++r) nb = regimes[r].n_stacks > nb ? regimes[r].n_stacks : nb;
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = ix->stream;
    if (stats) memset(stats, 0, sizeof *stats);
    if (n_jobs == 0) { *hits_out = (uint32_t *)calloc(9, 4); return 0; }

    // device staging: regimes | jobs | list | codes
    const size_t o_reg = 0, o_jobs = 256, o_list = o_jobs + ((size_t)n_jobs * sizeof(hsa_job_t) + 255) / 256 * 256;
    const size_t o_codes = o_list + ((size_t)n_jobs * 4 + 255) / 256 * 256;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, o_codes + codes_len + 256))) return rc;
    char *din = (char *)ix->d_in;
    HSA_HIP(hipMemcpyAsync(din + o_reg, regimes, sizeof(hsa_regime_t) * n_regimes, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, sizeof(hsa_job_t) * n_jobs, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(din + o_codes, codes, codes_len, hipMemcpyHostToDevice, st));
    // outputs: n_aln | flags | hit_off | hits
    uint64_t hit_cap = (uint64_t)n_jobs * 4 + 4096;
    const size_t o_fl = ((size_t)n_jobs * 4 + 255) / 256 * 256;
    const size_t o_ho = o_fl + ((size_t)n_jobs * 4 + 255) / 256 * 256;
    const size_t o_hits = o_ho + ((size_t)n_jobs * 8 + 255) / 256 * 256;
    if ((rc = hsa_grow(&ix->d_out, &ix->d_out_cap, o_hits + hit_cap * 36 + 256))) return rc;
    char *dout = (char *)ix->d_out;
    int32_t *d_n = (int32_t *)dout;
    uint32_t *d_fl = (uint32_t *)(dout + o_fl);
    uint64_t *d_ho = (uint64_t *)(dout + o_ho);
    uint32_t *d_hits = (uint32_t *)(dout + o_hits);
    unsigned long long *d_ctr = (unsigned long long *)ix->d_ctr;

    LaunchPlan P;
    if ((rc = plan_launch(ix, n_jobs, max_len, max_seed, nb, false, P))) return rc;
    HSA_HIP(hipEventRecord(ix->ev0, st));
    if ((rc = launch_pass(ix, P, ix->main, (const hsa_regime_t *)(din + o_reg), (const hsa_job_t *)(din + o_jobs),
                          nullptr, n_jobs, (const uint8_t *)(din + o_codes), d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, st)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    unsigned long long ctr[8];
    HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(n_aln, d_n, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(flags, d_fl, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(hit_off, d_ho, (size_t)n_jobs * 8, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    float ms = 0;
    HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    uint64_t total = ctr[1] < hit_cap ? ctr[1] : hit_cap;
    uint32_t *h = (uint32_t *)malloc((total + 1) * 36);
    if (total) HSA_HIP(hipMemcpy(h, d_hits, total * 36, hipMemcpyDeviceToHost));
    if (stats) {
        stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
        stats->kernel_ms += ms; stats->main_kernel_ms += ms; stats->main_launches += 1;
    }

    // overflowed reads: re-run with large per-read capacity (never a CPU path)
    for (int round = 0; round < 4; ++round) {
        int32_t *list = (int32_t *)malloc(sizeof(int32_t) * n_jobs);
        int n_over = 0;
        for (int j = 0; j < n_jobs; ++j) if (flags[j] & HSA_F_OVERFLOW) list[n_over++] = j;
        if (n_over == 0) { free(list); break; }
        if (stats) stats->overflow_reruns += n_over;
        LaunchPlan B;
        if ((rc = plan_launch(ix, n_over, max_len, max_seed, nb, true, B))) { free(list); free(h); return rc; }
        uint64_t cap2 = (uint64_t)n_over * 256 * (round + 1) + 65536;
        void *d2 = nullptr;
        size_t o2_fl = ((size_t)n_jobs * 4 + 255) / 256 * 256;
        size_t o2_ho = o2_fl * 2, o2_hits = o2_ho + ((size_t)n_jobs * 8 + 255) / 256 * 256;
        HSA_HIP(hipMalloc(&d2, o2_hits + cap2 * 36));
        HSA_HIP(hipMemcpyAsync(din + o_list, list, sizeof(int32_t) * n_over, hipMemcpyHostToDevice, st));
        char *c2 = (char *)d2;
        HSA_HIP(hipEventRecord(ix->ev0, st));
        if ((rc = launch_pass(ix, B, ix->big, (const hsa_regime_t *)(din + o_reg), (const hsa_job_t *)(din + o_jobs),
                              (const int32_t *)(din + o_list), n_over, (const uint8_t *)(din + o_codes), (int32_t *)c2,
                              (uint32_t *)(c2 + o2_fl), (uint64_t *)(c2 + o2_ho), (uint32_t *)(c2 + o2_hits), cap2,
                              d_ctr, st))) {
            free(list); free(h); (void)hipFree(d2); return rc;
        }
        HSA_HIP(hipEventRecord(ix->ev1, st));
        int32_t *n2 = (int32_t *)malloc((size_t)n_jobs * 4);
        uint32_t *f2 = (uint32_t *)malloc((size_t)n_jobs * 4);
        uint64_t *o2 = (uint64_t *)malloc((size_t)n_jobs * 8);
        HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(n2, c2, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(f2, c2 + o2_fl, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(o2, c2 + o2_ho, (size_t)n_jobs * 8, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipStreamSynchronize(st));
        HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
        uint64_t t2 = ctr[1] < cap2 ? ctr[1] : cap2;
        h = (uint32_t *)realloc(h, (total + t2 + 1) * 36);
        if (t2) HSA_HIP(hipMemcpy(h + total * 9, c2 + o2_hits, t2 * 36, hipMemcpyDeviceToHost));
        for (int q = 0; q < n_over; ++q) {
            int j = list[q];
            n_aln[j] = n2[j]; flags[j] = f2[j]; hit_off[j] = o2[j] + total;
        }
        total += t2;
        if (stats) {
            stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
            stats->kernel_ms += ms;
        }
        free(n2); free(f2); free(o2); free(list);
        (void)hipFree(d2);
    }
    for (int j = 0; j < n_jobs; ++j)
        if (flags[j] & HSA_F_OVERFLOW) { hsa_set_error("read %d exceeds the large-pass capacity", j); free(h); return HSA_E_ARG; }
    *hits_out = h;
    return (long)total;
}

extern "C" int hsa_search_device(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                                 const hsa_device_batch_t *b, void *stream)
{
    // regimes: host array; copied into the index's staging area
    int rc = check_regimes(regimes, n_regimes);
    if (rc) return rc;
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = stream ? (hipStream_t)stream : ix->stream;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, 1024))) return rc;
    HSA_HIP(hipMemcpyAsync(ix->d_in, regimes, sizeof(hsa_regime_t) * n_regimes, hipMemcpyHostToDevice, st));
    int nb = 0;
    for (int r = 0; r < n_regimes; ++r) nb = regimes[r].n_stacks > nb ? regimes[r].n_stacks : nb;
    LaunchPlan P;
    if ((rc = plan_launch(ix, b->n_jobs, 1023, 1023, nb, false, P))) return rc;
    return launch_pass(ix, P, ix->main, (const hsa_regime_t *)ix->d_in, b->d_jobs, nullptr, b->n_jobs, b->d_codes,
                       b->d_n_aln, b->d_flags, b->d_hit_off, b->d_hits, b->hit_cap,
                       (unsigned long long *)b->d_counters, st);
}
