#pragma once
// hsa_search_any.h -- the search for what k_search's fixed layouts cannot hold: reads
// longer than 1 023 bases, more gap opens than its 4-bit field counts (max_gapo > 14),
// max_diff > 125, more scores than its score table (n_stacks > 512) or more reachable
// scores than its bucket mask (> 128).  The reference accepts all of them
// (bwa_seq_t.len:19, bwtaln.h:96; the 16-bit read position in gap_entry_t.info,
// bwtgap.c:157), so the drop-in must too.
//
// k_search_any restates bwtgap.c:118-331 and bwtaln.c:303-373 one (read, strand) per
// lane with every piece of state in HBM, sized per call: the widths of the strand
// being searched (bwt_cal_width, computed when the strand is searched: rc, then fwd
// only if rc had no hit, bwtaln.c:343-359), one LIFO per score exactly as gap_stack_t
// (bwtgap.c:13-92: `best` and its upward rescan), entries linked in a per-lane pool
// whose popped slots are reused (live entries <= max_entries + 9, bwtgap.c:150-151),
// and the hits staged per lane.  Two capacity passes: every read with a modest pool,
// then the reads that overflowed it with pools up to the reference's own bound.
//
// Slow by design (no LDS, no batching of rare paths): these regimes and read lengths
// are rare, and the fast kernel serves everything else.  Parity: the same restatement
// as k_search, so the same oracle (tests/test_gpu_any.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ANY_NIL 0xFFFFFFFFu
#define ANY_MAX_LEN 65535          // gap_entry_t.info keeps the position in 16 bits (bwtgap.c:157)
#define ANY_MAX_STACKS 65536       // score LIFOs per regime (heads per lane in HBM)

// gap_entry_t (bwtaln.h:52-58): n_mm / n_gapo / n_gape are 8-bit fields there, so
// they wrap modulo 256 as in the reference
template <typename IT> struct AnyEnt {
    IT k, l, rk, rl;
    uint32_t info;                 // score << 21 | i, as gap_push writes it (bwtgap.c:60)
    uint8_t mm, go, ge, st;
    int32_t ldp;                   // last_diff_pos
};

struct AnyArgs {
    RankDir fwd, rev;
    RankDir64 fwd64, rev64;
    uint32_t T;
    uint64_t T64;
    uint32_t C[5];
    uint64_t C64[5];
    const hsa_regime_t *regimes;   // device copy, 1 or 2
    const hsa_job_t *jobs;
    const int32_t *list;           // the jobs of this pass (list positions 0 .. *n_dev)
    const unsigned long long *n_dev;
    int n_host;                    // or a host count when n_dev is null
    const uint8_t *codes;
    const hsa_mg_job_t *mg;        // caller-width mode (bwt_match_gap called directly)
    int32_t *cw;                   //   the caller's bwt_width_t pairs, updated in place (Q6)
    int32_t *n_aln;
    uint32_t *flags;
    uint64_t *hit_off;
    uint32_t *hits;
    uint64_t hit_cap;
    unsigned long long *ctr;       // the batch's statistics counters (include/hsa_gpu.h)
    unsigned long long *qhead;     // this pass's queue head
    int32_t *ovf_list;             // overflowed jobs for the next pass (count in *ovf_n), or null
    unsigned long long *ovf_n;
    // per-lane scratch: lane t's region starts at t * lane_bytes
    uint8_t *scratch;
    size_t lane_bytes;
    uint32_t nlanes;
    uint32_t max_len, max_seed, n_stacks_max, pcap, hcap;
    uint32_t o_ww, o_wb, o_sw, o_sb, o_heads, o_pool, o_link, o_hits;   // byte offsets in a lane's region
};

template <typename IT> struct AnyIx;
template <> struct AnyIx<uint32_t> {
    __device__ static const RankDir &fwd(const AnyArgs &a) { return a.fwd; }
    __device__ static const RankDir &rev(const AnyArgs &a) { return a.rev; }
    __device__ static uint32_t T(const AnyArgs &a) { return a.T; }
    __device__ static uint32_t C(const AnyArgs &a, uint32_t c) { return a.C[c]; }
};
template <> struct AnyIx<uint64_t> {
    __device__ static const RankDir64 &fwd(const AnyArgs &a) { return a.fwd64; }
    __device__ static const RankDir64 &rev(const AnyArgs &a) { return a.rev64; }
    __device__ static uint64_t T(const AnyArgs &a) { return a.T64; }
    __device__ static uint64_t C(const AnyArgs &a, uint32_t c) { return a.C64[c]; }
};

// Scratch layout of one lane for a pass (host and device agree through AnyArgs).
template <typename IT>
static size_t any_layout(AnyArgs &A, uint32_t max_len, uint32_t max_seed, uint32_t n_stacks, uint32_t pcap,
                         uint32_t hcap, uint32_t hw)
{
    auto al = [](size_t x) { return (x + 15) / 16 * 16; };
    size_t o = 0;
    A.o_ww = (uint32_t)o; o = al(o + sizeof(IT) * ((size_t)max_len + 1));
    A.o_wb = (uint32_t)o; o = al(o + 4 * ((size_t)max_len + 1));
    A.o_sw = (uint32_t)o; o = al(o + sizeof(IT) * ((size_t)max_seed + 1));
    A.o_sb = (uint32_t)o; o = al(o + 4 * ((size_t)max_seed + 1));
    A.o_heads = (uint32_t)o; o = al(o + 4 * (size_t)n_stacks);
    A.o_hits = (uint32_t)o; o = al(o + 4 * (size_t)hw * hcap);
    A.o_link = (uint32_t)o; o = al(o + 4 * (size_t)pcap);
    A.o_pool = (uint32_t)o; o = al(o + sizeof(AnyEnt<IT>) * (size_t)pcap);
    A.max_len = max_len; A.max_seed = max_seed; A.n_stacks_max = n_stacks; A.pcap = pcap; A.hcap = hcap;
    A.lane_bytes = o;
    return o;
}

template <typename IT>
__global__ void __launch_bounds__(64) k_search_any(AnyArgs a)
{
    using Ix = AnyIx<IT>;
    constexpr uint32_t OW = sizeof(IT) == 4 ? 9u : 14u;         // bwt_aln1_t / hsa_aln64_t words
    const size_t lane = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (lane >= a.nlanes) return;
    uint8_t *const base = a.scratch + lane * a.lane_bytes;
    IT *const ww = reinterpret_cast<IT *>(base + a.o_ww);        // width_back[].w
    int32_t *const wbid = reinterpret_cast<int32_t *>(base + a.o_wb);
    IT *const sw = reinterpret_cast<IT *>(base + a.o_sw);        // width_seed[].w
    int32_t *const sbid = reinterpret_cast<int32_t *>(base + a.o_sb);
    uint32_t *const heads = reinterpret_cast<uint32_t *>(base + a.o_heads);
    uint32_t *const hb = reinterpret_cast<uint32_t *>(base + a.o_hits);   // staged hits, 10 words each
    uint32_t *const link = reinterpret_cast<uint32_t *>(base + a.o_link);
    AnyEnt<IT> *const pool = reinterpret_cast<AnyEnt<IT> *>(base + a.o_pool);
    const IT TT = Ix::T(a);
    const uint64_t n_jobs = a.n_dev ? *a.n_dev : (uint64_t)a.n_host;
    // statistics: a read's work counts once, when it completes (a read this pass hands
    // to the large-capacity pass is counted there)
    uint64_t st_q = 0, st_wq = 0, st_fq = 0, st_b = 0, st_p = 0;
    uint64_t tq = 0, twq = 0, tfq = 0, tb = 0, tp = 0;

    for (;;) {
        const unsigned long long q = atomicAdd(a.qhead, 1ull);
        if (q >= n_jobs) break;
        const int job = a.list ? a.list[q] : (int)q;
        const hsa_job_t J = a.jobs[job];
        const hsa_regime_t R = a.regimes[J.regime & 1];
        const int len = (int)J.len;
        const uint8_t *const rd = a.codes + J.off;
        const hsa_mg_job_t *const M = a.mg ? a.mg + job : nullptr;
        // the pruning rows this call uses: the read's (width_back), and width_seed --
        // its own array, none, or width_back itself (bwtgap.c:809)
        const int seed_kind = M ? M->seed : ((int)len > J.seed_len ? HSA_SEED_OWN : HSA_SEED_NONE);
        const int slen = seed_kind == HSA_SEED_NONE ? 0 : J.seed_len;
        IT *const s_w = seed_kind == HSA_SEED_ALIAS ? ww : sw;
        int32_t *const s_b = seed_kind == HSA_SEED_ALIAS ? wbid : sbid;
        uint32_t fl = 0;
        int n_out = 0;
        uint64_t out_off = 0;
        bool done = false;

        for (int pass = 0; pass < 2 && !done; ++pass) {
            const int strand = M ? (M->strand & 1) : 1 - pass;   // rc first (bwtaln.c:343)
            if (M && pass > 0) break;
            // base p of the searched sequence: the read, or its reverse complement (a
            // direct bwt_match_gap call hands over the searched sequence itself)
            const bool rcs = strand && !M;
            auto seq = [&](int p) -> uint32_t {
                const uint32_t c = rd[rcs ? len - 1 - p : p];
                return rcs && c < 4 ? 3u - c : c;
            };
            // ---- widths (bwt_cal_width type 1, bwtaln.c:84-97); the caller's in mg mode
            if (M) {
                const int32_t *w = a.cw + 2 * M->wb_off;
                for (int t = 0; t <= len; ++t) { ww[t] = (IT)(uint32_t)w[2 * t]; wbid[t] = w[2 * t + 1]; }
                if (seed_kind == HSA_SEED_ALIAS && M->ws_off == HSA_MG_PREFIX) {   // a row's prefix: terminal
                    ww[len] = 0;
                    wbid[len] = (len ? wbid[len - 1] : 0) + 1;
                }
                if (seed_kind == HSA_SEED_OWN) {
                    const int32_t *v = a.cw + 2 * M->ws_off;
                    for (int t = 0; t <= slen; ++t) { sw[t] = (IT)(uint32_t)v[2 * t]; sbid[t] = v[2 * t + 1]; }
                }
            } else {
                auto width = [&](int n, int off, IT *w, int32_t *bid) {
                    IT k = 0, l = TT;
                    int b = 0;
                    for (int t = 0; t < n; ++t) {
                        const uint32_t c = seq(off + t);
                        if (c < 4) {                               // BWTSARangeForeward (2BWT-Interface.c:121)
                            IT ok, ol;
                            st_b += occ1_pair(Ix::rev(a), k, l + 1u, c, ok, ol);
                            k = Ix::C(a, c) + ok + 1u;
                            l = Ix::C(a, c) + ol;
                            st_q += 2; st_wq += 2;
                            if (strand == 0) st_fq += 2;
                        }
                        if (k > l || c > 3) { k = 0; l = TT; ++b; }
                        w[t] = l - k + 1u;
                        bid[t] = b;
                    }
                    w[n] = 0;
                    bid[n] = b + 1;
                };
                if (seed_kind == HSA_SEED_OWN) width(slen, len - slen, sw, sbid);   // bwtaln.c:344-346
                width(len, 0, ww, wbid);                                             // :348
            }

            // ---- bwt_match_gap (bwtgap.c:118-331)
            const int s_mm = R.s_mm, s_go = R.s_gapo, s_ge = R.s_gape, mode = R.mode;
            const int opt_max_diff = J.max_diff;
            auto score_of = [&](int mm, int go, int ge) { return mm * s_mm + go * s_go + ge * s_ge; };
            const int n_stacks = R.n_stacks;
            int best_score = score_of(opt_max_diff + 1, R.max_gapo + 1, R.max_gape + 1);
            int max_diff = opt_max_diff;
            int best_cnt = 0;
            long long best_cnt64 = 0;
            int n_aln = 0;
            // gap_stack_t: heads per score, best, n_entries; pool slots reused
            for (int s = 0; s < n_stacks; ++s) heads[s] = ANY_NIL;
            int best = n_stacks, n_entries = 0;
            uint32_t top = 0, free_head = ANY_NIL;
            bool ovf = false, err = false;
            auto push = [&](int i, IT k, IT l, IT rk, IT rl, int mm, int go, int ge, int st, int is_diff) {
                // the score from the arguments; the entry keeps 8-bit fields (bwtgap.c:53-66)
                const int score = score_of(mm, go, ge);
                const uint8_t m8 = (uint8_t)mm, g8 = (uint8_t)go, e8 = (uint8_t)ge;
                if (score < 0 || score >= n_stacks) { err = true; return; }      // undefined in the reference
                uint32_t slot;
                if (free_head != ANY_NIL) { slot = free_head; free_head = link[slot]; }
                else if (top < a.pcap) slot = top++;
                else { ovf = true; return; }
                AnyEnt<IT> &p = pool[slot];
                p.k = k; p.l = l; p.rk = rk; p.rl = rl;
                p.info = (uint32_t)score << 21 | (uint32_t)i;
                p.mm = m8; p.go = g8; p.ge = e8; p.st = (uint8_t)st;
                p.ldp = is_diff ? i : 0;
                link[slot] = heads[score];
                heads[score] = slot;
                ++n_entries;
                if (best > score) best = score;
            };
            push(len, 0, TT, 0, TT, 0, 0, 0, ST_M, 0);
            while (n_entries && !ovf && !err) {
                if (n_entries > R.max_entries) break;
                // gap_pop (bwtgap.c:77-92)
                const uint32_t slot = heads[best];
                const AnyEnt<IT> e = pool[slot];
                heads[best] = link[slot];
                link[slot] = free_head;
                free_head = slot;
                --n_entries;
                ++st_p;
                if (heads[best] == ANY_NIL && n_entries) {
                    int s = best + 1;
                    while (s < n_stacks && heads[s] == ANY_NIL) ++s;
                    best = s;
                } else if (n_entries == 0) {
                    best = n_stacks;
                }
                IT k = e.k, l = e.l, rk = e.rk, rl = e.rl;
                int i = (int)(e.info & 0xffffu);
                if (!(mode & MODE_NONSTOP) && (int)(e.info >> 21) > best_score + s_mm) break;
                int m = max_diff - (e.mm + e.go);
                if (mode & MODE_GAPE) m -= e.ge;
                if (m < 0) continue;
                int m_seed = 0;
                if (seed_kind != HSA_SEED_NONE) {
                    m_seed = R.max_seed_diff - (e.mm + e.go);
                    if (mode & MODE_GAPE) m_seed -= e.ge;
                }
                if (i > 0 && m < wbid[i - 1]) continue;
                bool hit = i == 0;
                if (!hit && m == 0 && (e.st == ST_M || (mode & MODE_GAPE) || e.ge == R.max_gape)) {
                    // bwt_match_exact (2BWT-Interface.c:365-388) with its write-back guard
                    IT xk = k, xl = l, xrl = rl;
                    bool ok = true;
                    for (int p = i - 1; p >= 0; --p) {
                        const uint32_t c = seq(p);
                        if (c > 3) { ok = false; break; }
                        IT oa[4], ob[4];
                        st_b += occ_pair(Ix::fwd(a), xk, xl + 1u, oa, ob);
                        st_q += 2;
                        IT oc = 0;
                        for (uint32_t d = c + 1; d < 4; ++d) oc += ob[d] - oa[d];
                        xk = Ix::C(a, c) + oa[c] + 1u;
                        xl = Ix::C(a, c) + ob[c];
                        xrl -= oc;
                        if (xk > xl) break;
                    }
                    if (!ok || xk > xl) continue;
                    const IT xrk = xrl - (xl - xk);
                    if (k) k = xk;
                    if (l) l = xl;
                    if (rk) rk = xrk;
                    if (rl) rl = xrl;
                    hit = true;
                }
                if (hit) {
                    const int score = score_of(e.mm, e.go, e.ge);
                    if (n_aln == 0) {
                        best_score = score;
                        int best_diff = e.mm + e.go;
                        if (mode & MODE_GAPE) best_diff += e.ge;
                        if (!(mode & MODE_NONSTOP)) max_diff = best_diff + 1 > opt_max_diff ? opt_max_diff : best_diff + 1;
                    }
                    if (sizeof(IT) == 4) {
                        if (score == best_score) best_cnt = (int)((uint32_t)best_cnt + (uint32_t)(l - k + 1u));
                        else if (best_cnt > R.max_top2) break;
                    } else {
                        if (score == best_score) best_cnt64 += (long long)(l - k + 1u);
                        else if (best_cnt64 > R.max_top2) break;
                    }
                    bool add = true;
                    if (e.go) {
                        for (int j = 0; j < n_aln; ++j) {
                            const uint32_t *h = hb + (size_t)j * 10;
                            const IT hk = sizeof(IT) == 4 ? (IT)h[1] : (IT)((uint64_t)h[1] | (uint64_t)h[2] << 32);
                            const IT hl = sizeof(IT) == 4 ? (IT)h[2] : (IT)((uint64_t)h[3] | (uint64_t)h[4] << 32);
                            if (hk == k && hl == l) { add = false; break; }
                        }
                    }
                    if (add) {
                        if ((uint32_t)n_aln >= a.hcap) { ovf = true; break; }
                        // gap_shadow (bwtgap.c:94-105) on width_back
                        const IT x = l - k + 1u;
                        for (int p = 0, jj = 0; p < e.ldp; ++p) {
                            if (ww[p] > x) ww[p] -= x;
                            else if (ww[p] == x) { wbid[p] = 1; ww[p] = TT - (IT)(++jj); }
                        }
                        uint32_t *h = hb + (size_t)n_aln * 10;
                        h[0] = (uint32_t)e.mm | (uint32_t)e.go << 16 | (uint32_t)e.ge << 24;
                        if (sizeof(IT) == 4) {
                            h[1] = (uint32_t)k; h[2] = (uint32_t)l; h[3] = (uint32_t)rk; h[4] = (uint32_t)rl;
                        } else {
                            h[1] = (uint32_t)k; h[2] = (uint32_t)((uint64_t)k >> 32);
                            h[3] = (uint32_t)l; h[4] = (uint32_t)((uint64_t)l >> 32);
                            h[5] = (uint32_t)rk; h[6] = (uint32_t)((uint64_t)rk >> 32);
                            h[7] = (uint32_t)rl; h[8] = (uint32_t)((uint64_t)rl >> 32);
                        }
                        h[9] = (uint32_t)score;
                        ++n_aln;
                    }
                    continue;
                }
                // ---- expansion (bwtgap.c:245-325)
                --i;
                IT sk[4], sl[4], srk[4], srl[4];
                {
                    IT oa[4], ob[4];
                    st_b += occ_pair(Ix::fwd(a), k, l + 1u, oa, ob);
                    st_q += 2;
                    IT oc = 0;                                   // 2BWT-Interface.c:235-272
                    for (int c = 3; c >= 0; --c) {
                        sk[c] = Ix::C(a, c) + oa[c] + 1u;
                        sl[c] = Ix::C(a, c) + ob[c];
                        srl[c] = rl - oc;
                        srk[c] = srl[c] - (sl[c] - sk[c]);
                        oc += ob[c] - oa[c];
                    }
                }
                const IT occ = l - k + 1u;
                bool allow_diff = true, allow_M = true;
                if (i > 0) {
                    const int ii = i - (len - slen);
                    if (wbid[i - 1] > m - 1) allow_diff = false;
                    else if (wbid[i - 1] == m - 1 && wbid[i] == m - 1 && ww[i - 1] == ww[i]) allow_M = false;
                    if (seed_kind != HSA_SEED_NONE && ii > 0) {
                        if (s_b[ii - 1] > m_seed - 1) allow_diff = false;
                        else if (s_b[ii - 1] == m_seed - 1 && s_b[ii] == m_seed - 1 && s_w[ii - 1] == s_w[ii]) allow_M = false;
                    }
                }
                const int tmp = (mode & MODE_LOGGAP) ? int_log2((uint32_t)(e.ge + e.go)) / 2 + 1 : e.go + e.ge;
                if (allow_diff && i >= R.indel_end_skip + tmp && len - i >= R.indel_end_skip + tmp) {
                    if (e.st == ST_M) {
                        if (e.go < R.max_gapo) {
                            push(i, k, l, rk, rl, e.mm, e.go + 1, e.ge, ST_I, 1);
                            for (int j = 0; j < 4; ++j)
                                if (sk[j] <= sl[j]) push(i + 1, sk[j], sl[j], srk[j], srl[j], e.mm, e.go + 1, e.ge, ST_D, 1);
                        }
                    } else if (e.st == ST_I) {
                        if (e.ge < R.max_gape) push(i, k, l, rk, rl, e.mm, e.go, e.ge + 1, ST_I, 1);
                    } else if (e.st == ST_D) {
                        if (e.ge < R.max_gape && (e.ge + e.go < max_diff || occ < (IT)R.max_del_occ))
                            for (int j = 0; j < 4; ++j)
                                if (sk[j] <= sl[j]) push(i + 1, sk[j], sl[j], srk[j], srl[j], e.mm, e.go, e.ge + 1, ST_D, 1);
                    }
                }
                const uint32_t si = seq(i);
                if (allow_diff && allow_M) {
                    for (int j = 1; j <= 4; ++j) {
                        const uint32_t c = (si + (uint32_t)j) & 3u;
                        const int is_mm = (j != 4 || si > 3);
                        if (sk[c] <= sl[c]) push(i, sk[c], sl[c], srk[c], srl[c], e.mm + is_mm, e.go, e.ge, ST_M, is_mm);
                    }
                } else if (si < 4) {
                    if (sk[si] <= sl[si]) push(i, sk[si], sl[si], srk[si], srl[si], e.mm, e.go, e.ge, ST_M, 0);
                }
            }
            if (err) { atomicAdd(&a.ctr[5], 1ull); fl = HSA_F_OVERFLOW; done = true; break; }
            if (ovf) { fl = HSA_F_OVERFLOW; done = true; break; }
            if (M && !(seed_kind == HSA_SEED_ALIAS && M->ws_off == HSA_MG_PREFIX)) {   // width_back back (Q6)
                int32_t *w = a.cw + 2 * M->wb_off;
                for (int t = 0; t <= len; ++t) { w[2 * t] = (int32_t)(uint32_t)ww[t]; w[2 * t + 1] = wbid[t]; }
            }
            if (n_aln > 0 || M) {
                if (n_aln > 0) {
                    const unsigned long long o = atomicAdd(&a.ctr[1], (unsigned long long)n_aln);
                    if (o + (uint64_t)n_aln > a.hit_cap) { fl = HSA_F_OVERFLOW; done = true; break; }
                    uint32_t *dst = a.hits + o * OW;
                    for (int h = 0; h < n_aln; ++h) {
                        const uint32_t *v = hb + (size_t)h * 10;
                        const uint32_t end = h == 0 && !M ? (uint32_t)(len - 1) : 0u;   // bwtaln.c:371-372
                        if (sizeof(IT) == 4) {
                            dst[h * 9 + 0] = v[0]; dst[h * 9 + 1] = v[1]; dst[h * 9 + 2] = v[2];
                            dst[h * 9 + 3] = v[3]; dst[h * 9 + 4] = v[4];
                            dst[h * 9 + 5] = (uint32_t)strand << 30; dst[h * 9 + 6] = 0;
                            dst[h * 9 + 7] = end; dst[h * 9 + 8] = v[9];
                        } else {
                            dst[h * 14 + 0] = v[0]; dst[h * 14 + 1] = (uint32_t)strand << 30;
                            for (int j = 1; j < 9; ++j) dst[h * 14 + 1 + j] = v[j];
                            dst[h * 14 + 10] = 0; dst[h * 14 + 11] = end; dst[h * 14 + 12] = v[9];
                            dst[h * 14 + 13] = 0;
                        }
                    }
                    out_off = o;
                }
                n_out = n_aln;
                done = true;
            }
        }
        if (!done) fl = HSA_F_FALLBACK;                  // no hit on either strand
        if (fl & HSA_F_OVERFLOW) {
            n_out = 0; out_off = 0;
            if (a.ovf_list) a.ovf_list[atomicAdd(a.ovf_n, 1ull)] = job;
            else atomicAdd(&a.ctr[11], 1ull);
        }
        a.n_aln[job] = n_out;
        a.flags[job] = fl;
        a.hit_off[job] = out_off;
        if (!(fl & HSA_F_OVERFLOW)) { tq += st_q; twq += st_wq; tfq += st_fq; tb += st_b; tp += st_p; }
        st_q = st_wq = st_fq = st_b = st_p = 0;
    }
    st_q = tq; st_wq = twq; st_fq = tfq; st_b = tb; st_p = tp;
    atomicAdd(&a.ctr[2], (unsigned long long)st_q);
    atomicAdd(&a.ctr[3], (unsigned long long)st_b);
    atomicAdd(&a.ctr[4], (unsigned long long)st_p);
    atomicAdd(&a.ctr[7], (unsigned long long)st_wq);
    atomicAdd(&a.ctr[13], (unsigned long long)st_fq);
    atomicAdd(&a.ctr[14], (unsigned long long)st_fq);
}
