// nw_quant.hip -- indel / substitution quantification of aligned reads on gfx950,
// and its C ABI (include/crispr_quant.h).
//
// Replaces process_df_chunk (CRISPRessoCORE.py:428-753), which walks a DataFrame
// row by row in Python: regex runs of '.' / '-' over the three alignment strings,
// ref_positions lookups (CORE:2055-2067), set intersections with INCLUDE_IDXS /
// EXON_POSITIONS / SPLICING_POSITIONS and numpy fancy-index increments of fifteen
// per-position vectors.
//
// One wave per read, 256 alignment columns per step (4 per lane, dword loads of
// the three rows).  Per step: base-count prefix (amplicon index of every column)
// and run boundaries from ballots + mbcnt; substitution positions and deletion
// run ids are written into a per-wave position array in LDS, run records
// (deletion: first position, size, window/exon/splice hits from prefix counts;
// insertion: the two flank positions of CORE:520-526) into per-wave run lists.
// A run pass classifies the read (HDR / MIXED / NHEJ / UNMODIFIED, CORE:530-575),
// applies the NHEJ window filter with the reference's quirks (CORE:611-641) and
// the frameshift analysis (CORE:653-725); a position pass then adds the read's
// contributions to the block's LDS copy of the vectors -- once per distinct
// position, which is what numpy's buffered `vec[idx] += 1` does -- and clears the
// position array for the next read.  Blocks write their vectors to a partial
// slab; a second kernel sums the slabs into int64 totals.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crispr_nw.h"
#include "../../include/crispr_quant.h"
#include "nw_common.h"
#include "nw_edna.h"

namespace nwq {

enum : int { V_INS, V_DEL, V_MUT, V_ANY, V_INS_MIX, V_DEL_MIX, V_MUT_MIX, V_INS_HDR, V_DEL_HDR, V_MUT_HDR,
             V_INS_NC, V_DEL_NC, V_MUT_NC, V_AVG_DEL, V_AVG_INS, NV };
enum : int { C_FS, C_NONFS, C_NONMOD, C_SPLICE };
enum : unsigned { F_IGN_SUB = 1, F_IGN_INS = 2, F_IGN_DEL = 4, F_HIDE = 8, F_FRAMESHIFT = 16, F_NFIX = 32 };
enum : unsigned { T_INC = 1, T_EXON = 2, T_SPL = 4 };                 // position table bits
enum : unsigned { P_SUB = 1, P_INS = 2 };                              // position marks; bits 16+: del run + 1
enum : int { R_INC = 1, R_EXON = 2, R_SPL = 4, R_KEPT = 8, R_POST = 16 };   // run flags

typedef short run4 __attribute__((ext_vector_type(4)));   // deletion {pos, size, flags, exon count}
                                                          // insertion {flank a, flank b, size, flags}
struct QArgs {
    uint8_t* aln;
    int64_t stride;
    const int32_t* len;
    int64_t len_stride;
    const uint8_t* pre;
    int64_t n;
    int4* out;
    uint32_t* partial;       // [gridDim.x][nwords]
    const int32_t* prefix;   // [3][LEN + 1] prefix counts of INC / EXON / SPL, then [LEN] table bytes
    const int32_t* list;     // reads to process (quant_lanes' fallback list), or null: reads [0, n)
    const int32_t* list_count;
    int32_t LEN, H, run_cap, window, nwords, wave_words, base_words;
    uint32_t flags;
};


__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ bool wave_any(bool p) { return ballot(p) != 0ull; }

// Inclusive prefix sum over the 64 lanes on DPP (row_shr 1/2/3 of the input,
// row_shr 4/8 within rows, row_bcast 15/31 across rows): 7 adds, no LDS.
template <int CTRL, int ROWS, int BANKS>
__device__ __forceinline__ unsigned dpp_mov(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, BANKS, false);
}
__device__ __forceinline__ unsigned wave_scan_incl(unsigned v) {
    unsigned s = v + dpp_mov<0x111, 0xf, 0xf>(v);
    s += dpp_mov<0x112, 0xf, 0xf>(v);
    s += dpp_mov<0x113, 0xf, 0xf>(v);
    s += dpp_mov<0x114, 0xf, 0xe>(s);
    s += dpp_mov<0x118, 0xf, 0xc>(s);
    s += dpp_mov<0x142, 0xa, 0xf>(s);
    s += dpp_mov<0x143, 0xc, 0xf>(s);
    return s;
}
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) { return ~nw::wave_max_u32(~v); }

__device__ __forceinline__ void vadd(uint32_t* h, int v, int LEN, unsigned x) {
    if (x) atomicAdd(h + v * LEN, x);
}

// Column step state carried between 256-column steps of one read.
struct Carry {
    int B;                  // amplicon bases before the step
    int ds, de, is, ie;     // deletion / insertion run starts / ends so far
    int prev;               // gap state of the column before the step (bit0 read gap, bit1 amplicon gap)
};

__global__ __launch_bounds__(512) void quant_kernel(QArgs a) {
    extern __shared__ uint32_t smem[];
    const int LEN = a.LEN;
    uint32_t* blk = smem;                                // vectors, counters, histograms
    int32_t* incp = (int32_t*)(blk + a.nwords);
    int32_t* exop = incp + (LEN + 1);
    int32_t* splp = exop + (LEN + 1);
    uint8_t* tbl = (uint8_t*)(splp + (LEN + 1));
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    uint32_t* posw = smem + a.base_words + wave * a.wave_words;
    run4* druns = (run4*)(posw + ((LEN + 1) & ~1));
    run4* iruns = druns + a.run_cap;

    for (int i = threadIdx.x; i < a.nwords; i += blockDim.x) blk[i] = 0;
    const int pref_words = 3 * (LEN + 1) + (LEN + 3) / 4;
    for (int i = threadIdx.x; i < pref_words; i += blockDim.x) incp[i] = a.prefix[i];
    for (int i = threadIdx.x; i < wpb * a.wave_words; i += blockDim.x) smem[a.base_words + i] = 0;
    __syncthreads();

    const unsigned flags = a.flags;
    const bool nfix = flags & F_NFIX;
    const bool hide = flags & F_HIDE;
    const unsigned ign_sub = (flags & F_IGN_SUB) ? 0u : 0xfu;
    const unsigned ign_ins = (flags & F_IGN_INS) ? 0u : 0xfu;
    const unsigned ign_del = (flags & F_IGN_DEL) ? 0u : 0xfu;
    uint32_t* ctr = blk + NV * LEN;
    uint32_t* hin = ctr + 4;
    uint32_t* hfs = hin + a.H;
    const int64_t stride = a.stride;

    // Reads go to waves in groups of 64: one coalesced load of the flags and
    // lengths, one coalesced store of the results; rows of the next read to
    // process are loaded while the current one is worked on.
    // A work list (quant_lanes' fallback reads: a few dozen per 1M) goes one read per wave, not 64:
    // a wave works through its group's reads one after another.
    const int64_t n_eff = a.list ? (int64_t)*a.list_count : a.n;
    const int gsz = a.list ? 1 : 64;
    const int64_t ngroups = (n_eff + gsz - 1) / gsz;
    const int64_t tw = (int64_t)gridDim.x * wpb;
    for (int64_t grp = (int64_t)blockIdx.x * wpb + wave; grp < ngroups; grp += tw) {
        const int64_t pos = grp * gsz + lane;
        const bool valid = lane < gsz && pos < n_eff;
        const int32_t ridx = valid ? (a.list ? a.list[pos] : (int32_t)pos) : 0;
        const int64_t idx = ridx;
        const unsigned mypre = valid ? (unsigned)a.pre[idx] : (unsigned)NWQ_PRE_UNMODIFIED;
        const int mylen = valid ? a.len[idx * a.len_stride] : 1;
        const bool skip = (mypre & NWQ_PRE_UNMODIFIED) && !nfix;
        const bool badlen = mylen <= 0 || mylen > stride;
        int4 myout = make_int4((!skip && badlen) ? -1 : 0, 0, 0, 0);
        unsigned long long todo = ballot(!skip && !badlen);

        auto row_ptr = [&](int k) { return a.aln + (int64_t)__builtin_amdgcn_readlane(ridx, k) * 3 * stride; };
        auto load3 = [&](int k, int L, int c0, uint32_t& dr, uint32_t& dm, uint32_t& ds) {
            dr = dm = ds = 0;
            if (c0 < L) {
                const uint8_t* p = row_ptr(k) + c0;
                dr = *(const uint32_t*)p;
                dm = *(const uint32_t*)(p + stride);
                ds = *(const uint32_t*)(p + 2 * stride);
            }
        };
        uint32_t nr = 0, nm = 0, ns = 0;
        if (todo) {
            const int k = __builtin_ctzll(todo);
            load3(k, __builtin_amdgcn_readlane(mylen, k), 4 * lane, nr, nm, ns);
        }
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const unsigned pre = (unsigned)__builtin_amdgcn_readlane((int)mypre, k);
            const int L = __builtin_amdgcn_readlane(mylen, k);
            uint32_t dr = nr, dm = nm, ds = ns;
            if (todo) {
                const int k2 = __builtin_ctzll(todo);
                load3(k2, __builtin_amdgcn_readlane(mylen, k2), 4 * lane, nr, nm, ns);
            }
            uint8_t* Mrow = row_ptr(k) + stride;
            const unsigned f0 = (nfix && (__builtin_amdgcn_readlane((int)dr, 0) & 255) == 'N')
                                    ? (unsigned)'|' : (unsigned)(__builtin_amdgcn_readlane((int)dm, 0) & 255);
            Carry cy{0, 0, 0, 0, 0, 0};
            unsigned nsub = 0, nsub_inc = 0, subbits = 0;   // subbits: 1 exon, 2 splice, 4 exon&inc, 8 splice&inc
            int pmin = LEN, pmax = -1;                       // range of positions marked in posw
            bool neq = false, oob = false;
            for (int cb = 0; cb <= L; cb += 256) {
                const int c0 = cb + 4 * lane;
                if (cb) load3(k, L, c0, dr, dm, ds);
                unsigned isb = 0, gR = 0, gS = 0, dot = 0;
                uint32_t dmf = dm;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (c0 + q >= L) break;
                    const unsigned rc = (dr >> (8 * q)) & 255u, sc = (ds >> (8 * q)) & 255u;
                    unsigned mc = (dm >> (8 * q)) & 255u;
                    const bool base = rc == 'A' || rc == 'C' || rc == 'G' || rc == 'T' || rc == 'N';
                    isb |= (unsigned)base << q;
                    gR |= (unsigned)(rc == '-') << q;
                    gS |= (unsigned)(sc == '-') << q;
                    if (nfix && rc == 'N') {
                        mc = '|';
                        dmf = (dmf & ~(255u << (8 * q))) | ((unsigned)'|' << (8 * q));
                    }
                    dot |= (unsigned)(mc == '.') << q;
                    neq |= mc != f0;
                }
                if (nfix && dmf != dm) *(uint32_t*)(Mrow + c0) = dmf;
                gR &= ign_ins;
                gS &= ign_del;
                dot &= ign_sub;
                // gap state of the column before this lane's first one
                const int st = (int)(((gS >> 3) & 1u) | (((gR >> 3) & 1u) << 1));
                const int pl = nw::shr1(st, cy.prev);
                const unsigned pS = ((gS << 1) | (unsigned)(pl & 1)) & 0xfu;
                const unsigned pR = ((gR << 1) | (unsigned)((pl >> 1) & 1)) & 0xfu;
                const unsigned dstart = gS & ~pS, dend = ~gS & pS & 0xfu;
                const unsigned istart = gR & ~pR, iend = ~gR & pR & 0xfu;

                // lane prefixes of (bases, del starts, del ends) and (ins starts, ins ends), packed
                const unsigned va = (unsigned)__popc(isb) | ((unsigned)__popc(dstart) << 9) |
                                    ((unsigned)__popc(dend) << 17);
                const unsigned vb = (unsigned)__popc(istart) | ((unsigned)__popc(iend) << 8);
                const unsigned sa = wave_scan_incl(va), sb = wave_scan_incl(vb);
                const unsigned ea = sa - va, eb = sb - vb;
                const int Bl = cy.B + (int)(ea & 511u);
                const int dsp = cy.ds + (int)((ea >> 9) & 255u);
                const int dep = cy.de + (int)((ea >> 17) & 255u);
                const int isp = cy.is + (int)(eb & 255u);
                const int iep = cy.ie + (int)((eb >> 8) & 255u);

                // starts, deletion marks, substitutions
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned lt = (1u << q) - 1u, bit = 1u << q;
                    const int Bk = Bl + __popc(isb & lt);
                    if (dstart & bit) druns[dsp + __popc(dstart & lt)].x = (short)Bk;
                    if (gS & bit) {
                        const int jr = dsp + __popc(dstart & (lt | bit)) - 1;
                        if (Bk < LEN) {
                            posw[Bk] = (uint32_t)(jr + 1) << 16;
                            pmin = min(pmin, Bk);
                            pmax = max(pmax, Bk);
                        } else {
                            oob = true;
                        }
                    }
                    if (istart & bit) iruns[isp + __popc(istart & lt)].x = (short)(c0 + q);
                    if (dot & bit) {
                        if (Bk < LEN) {
                            posw[Bk] = P_SUB;
                            pmin = min(pmin, Bk);
                            pmax = max(pmax, Bk);
                            const unsigned t = tbl[Bk];
                            ++nsub;
                            nsub_inc += t & T_INC;
                            subbits |= ((t & T_EXON) ? 1u : 0u) | ((t & T_SPL) ? 2u : 0u);
                            if (t & T_INC) subbits |= ((t & T_EXON) ? 4u : 0u) | ((t & T_SPL) ? 8u : 0u);
                        } else {
                            oob = true;
                        }
                    }
                }
                // ends (their starts are in LDS by now: one wave, in-order LDS queue)
                if (dend | iend) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const unsigned lt = (1u << q) - 1u, bit = 1u << q;
                        const int Bk = Bl + __popc(isb & lt);
                        if ((dend & bit) && Bk <= LEN) {
                            const int j = dep + __popc(dend & lt);
                            const int ps = druns[j].x;
                            const int f = (incp[Bk] - incp[ps] > 0 ? R_INC : 0) |
                                          (splp[Bk] - splp[ps] > 0 ? R_SPL : 0);
                            druns[j] = run4{(short)ps, (short)(Bk - ps), (short)f, (short)(exop[Bk] - exop[ps])};
                        }
                        if ((iend & bit) && Bk <= LEN) {
                            const int j = iep + __popc(iend & lt);
                            const int c = c0 + q;
                            const int s0 = iruns[j].x;
                            const int fa = s0 > 0 ? Bk - 1 : -1;
                            const int fb = c < L ? Bk : (Bk > 0 ? -Bk : -1);
                            int f = 0;     // T_* and R_INC / R_EXON / R_SPL share bit positions
                            if (fa >= 0 && fa < LEN) f |= tbl[fa];
                            if (fb >= 0 && fb < LEN) f |= tbl[fb];
                            iruns[j] = run4{(short)fa, (short)fb, (short)(c - s0), (short)f};
                        }
                    }
                }
                const unsigned ta = (unsigned)__builtin_amdgcn_readlane((int)sa, 63);
                const unsigned tb = (unsigned)__builtin_amdgcn_readlane((int)sb, 63);
                cy.B += (int)(ta & 511u);
                cy.ds += (int)((ta >> 9) & 255u);
                cy.de += (int)((ta >> 17) & 255u);
                cy.is += (int)(tb & 255u);
                cy.ie += (int)((tb >> 8) & 255u);
                cy.prev = __builtin_amdgcn_readlane(st, 63);
            }
            const int nds = cy.ds, nis = cy.is;

            const bool bad = cy.B != LEN || wave_any(oob);
            const bool unmod = (pre & NWQ_PRE_UNMODIFIED) || (nfix && !wave_any(neq));
            const bool counting = !bad && !unmod;
            int cls = 0, n_mut = 0, n_ins = 0, n_del = 0;
            bool windowed = false, noncoding = false;
            if (counting) {
                const int nsub_t = (int)nw::wave_sum_u32(nsub), nsubi_t = (int)nw::wave_sum_u32(nsub_inc);
                bool hit_l = false;
                for (int j = lane; j < nds; j += 64) hit_l |= (druns[j].z & R_INC) != 0;
                for (int j = lane; j < nis; j += 64) hit_l |= (iruns[j].w & R_INC) != 0;
                const bool hit = nsubi_t > 0 || wave_any(hit_l);
                cls = (pre & NWQ_PRE_HDR) ? 2 : (pre & NWQ_PRE_MIXED) ? 3 : hit ? 1 : 0;
                windowed = cls == 1 && a.window != 0;

                bool kept_l = false;
                for (int j = lane; j < nds; j += 64) kept_l |= !windowed || (druns[j].z & R_INC);
                const bool post_sel = windowed && wave_any(kept_l);
                int ndel_l = 0, exdel_l = 0;
                bool spldel_l = false;
                for (int j = lane; j < nds; j += 64) {
                    run4 d = druns[j];
                    const bool kept = !windowed || (d.z & R_INC);
                    const bool post = post_sel ? kept : true;
                    d.z |= (kept ? R_KEPT : 0) | (post ? R_POST : 0);
                    druns[j] = d;
                    ndel_l += kept ? d.y : 0;
                    exdel_l += post ? d.w : 0;
                    spldel_l |= post && (d.z & R_SPL);
                }
                int nins_l = 0, insex_len_l = 0;
                bool insex_l = false, insspl_l = false;
                for (int j = lane; j < nis; j += 64) {
                    const run4 e = iruns[j];
                    const bool kept = !windowed || (e.w & R_INC);
                    const int wa = e.x < 0 ? e.x + LEN : e.x, wb = e.y < 0 ? e.y + LEN : e.y;
                    atomicOr(posw + wa, P_INS);
                    atomicOr(posw + wb, P_INS);
                    pmin = min(pmin, min(wa, wb));
                    pmax = max(pmax, max(wa, wb));
                    insspl_l |= (e.w & R_SPL) != 0;
                    if (kept) {
                        nins_l += e.z;
                        if (e.w & R_EXON) { insex_l = true; insex_len_l += e.z; }
                        if (cls != 0) {
                            atomicAdd(blk + V_AVG_INS * LEN + wa, (unsigned)e.z);
                            if (wb != wa) atomicAdd(blk + V_AVG_INS * LEN + wb, (unsigned)e.z);
                        }
                    }
                }
                n_mut = windowed ? nsubi_t : nsub_t;
                n_ins = nw::wave_sum(nins_l);
                n_del = nw::wave_sum(ndel_l);
                if ((flags & F_FRAMESHIFT) && cls != 0) {
                    const unsigned sb = (wave_any(subbits & 1u) ? 1u : 0u) | (wave_any(subbits & 2u) ? 2u : 0u) |
                                        (wave_any(subbits & 4u) ? 4u : 0u) | (wave_any(subbits & 8u) ? 8u : 0u);
                    const bool sub_exon = windowed ? (sb & 4u) : (sb & 1u);
                    const bool sub_spl = windowed ? (sb & 8u) : (sb & 2u);
                    const int exdel = nw::wave_sum(exdel_l);
                    const bool insex = wave_any(insex_l);
                    const int eff = nw::wave_sum(insex_len_l) - exdel;
                    const bool exon_mod = insex || exdel > 0 || sub_exon;
                    const bool has_lens = insex || exdel > 0;
                    const bool spliced = sub_spl || wave_any(spldel_l) || wave_any(insspl_l);
                    if (lane == 0) {
                        if (spliced) atomicAdd(ctr + C_SPLICE, 1u);
                        if (exon_mod) {
                            if (!has_lens) {
                                atomicAdd(ctr + C_NONFS, 1u);
                                atomicAdd(hin + LEN, 1u);
                            } else if (eff % 3 == 0) {
                                atomicAdd(ctr + C_NONFS, 1u);
                                atomicAdd(hin + LEN + eff, 1u);
                            } else {
                                atomicAdd(ctr + C_FS, 1u);
                                atomicAdd(hfs + LEN + eff, 1u);
                            }
                        } else {
                            atomicAdd(ctr + C_NONMOD, 1u);
                        }
                    }
                    noncoding = !exon_mod;
                }
            }

            // position pass over the marked range: the read's per-position vector
            // increments (once per distinct position); clears the marks
            const int lo = (int)wave_min_u32((unsigned)pmin);
            const int hi = (int)nw::wave_max_u32((unsigned)(pmax + 1)) - 1;
            for (int p = lo + lane; p <= hi; p += 64) {
                const uint32_t w = posw[p];
                if (!w) continue;
                posw[p] = 0;
                if (!counting) continue;
                const unsigned sub = w & P_SUB, ins = (w >> 1) & 1u;
                const int dj = (int)(w >> 16);
                int rf = 0, dsz = 0;
                if (dj) {
                    const run4 d = druns[dj - 1];
                    rf = d.z;
                    dsz = d.y;
                }
                const unsigned del = dj ? 1u : 0u;
                const unsigned sub_post = (sub && (!windowed || (tbl[p] & T_INC))) ? 1u : 0u;
                const unsigned del_post = (del && (rf & R_POST)) ? 1u : 0u;
                uint32_t* h = blk + p;
                if (cls == 3) {
                    vadd(h, V_MUT_MIX, LEN, sub); vadd(h, V_DEL_MIX, LEN, del); vadd(h, V_INS_MIX, LEN, ins);
                } else if (cls == 2) {
                    vadd(h, V_MUT_HDR, LEN, sub); vadd(h, V_DEL_HDR, LEN, del); vadd(h, V_INS_HDR, LEN, ins);
                } else if (cls == 1) {
                    vadd(h, V_MUT, LEN, hide ? sub_post : sub);
                    vadd(h, V_DEL, LEN, hide ? del_post : del);
                    vadd(h, V_INS, LEN, ins);
                }
                vadd(h, V_ANY, LEN, 1u);
                if (noncoding) {
                    vadd(h, V_MUT_NC, LEN, sub_post); vadd(h, V_DEL_NC, LEN, del_post); vadd(h, V_INS_NC, LEN, ins);
                }
                if (cls != 0 && del && (rf & R_KEPT)) vadd(h, V_AVG_DEL, LEN, (unsigned)dsz);
            }
            // counts are written only for rows left modified (CORE:651-660)
            if (lane == k) myout = cls ? make_int4(cls, n_mut, n_ins, n_del) : make_int4(bad ? -1 : 0, 0, 0, 0);
        }
        if (valid) a.out[idx] = myout;
    }

    __syncthreads();
    uint32_t* dst = a.partial + (int64_t)blockIdx.x * a.nwords;
    for (int i = threadIdx.x; i < a.nwords; i += blockDim.x) dst[i] = blk[i];
}

// Sum of the per-block slabs: blockIdx.y takes a contiguous slice of the slabs,
// adds into the (zeroed) int64 totals.
// Rows of one read rebuilt from its traceback runs (the aligner's device-resident ops
// output), exactly as the aligner writes them in NW_OUT_ROWS mode and nw_expand_ops does
// on the host (nw_expand.cpp): one wave per read, the three rows assembled in LDS (a
// run's columns spread over the lanes), then copied out as dwords.  Only the reads the
// quantification loads: not UNMODIFIED on input, unless the amplicon has N (nfix), and
// not empty.
__global__ __launch_bounds__(256) void expand_rows(const uint32_t* __restrict__ ops, const int64_t* ops_off,
                                                   const int32_t* stats, const uint8_t* reads, const int64_t* offsets,
                                                   int64_t bias, const uint8_t* amp, const uint32_t* rowpos,
                                                   const uint8_t* lut, int La, const uint8_t* pre, int all, int64_t n,
                                                   uint8_t* aln, int64_t stride, const int32_t* list,
                                                   const int32_t* list_count) {
    extern __shared__ uint8_t ex_sm[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    uint8_t* rows = ex_sm + (size_t)wave * 3 * stride;
    const int64_t n_eff = list ? (int64_t)*list_count : n;   // list: quant_lanes' fallback reads
    for (int64_t i = (int64_t)blockIdx.x * wpb + wave; i < n_eff; i += (int64_t)gridDim.x * wpb) {
        const int64_t r = list ? (int64_t)list[i] : i;
        const int L = __builtin_amdgcn_readfirstlane(stats[r * 8]);   // aln_len
        const unsigned pf = (unsigned)__builtin_amdgcn_readfirstlane((int)pre[r]);
        if (L <= 0 || L > stride || (!all && (pf & NWQ_PRE_UNMODIFIED))) continue;
        const int64_t k0 = ops_off[r], k1 = ops_off[r + 1];
        const uint8_t* rd = reads + (offsets[r] - bias);
        int col = 0, ia = 0, jb = 0;
        for (int64_t k = k0; k < k1; ++k) {
            const unsigned op = (unsigned)__builtin_amdgcn_readfirstlane((int)ops[k]);
            const int type = (int)(op >> 28), len = (int)(op & 0x0fffffffu);
            if (col + len > L) break;   // (not reached: the runs cover aln_len columns)
            for (int p = lane; p < len; p += 64) {
                uint8_t c0, c1, c2;
                if (type == 0) {
                    const uint8_t ca = amp[ia + p], cb = rd[jb + p];
                    uint8_t mk = '|';
                    if (ca != cb || ca == '-') {
                        const uint8_t ua = (ca >= 'a' && ca <= 'z') ? ca - 32 : ca;
                        const uint8_t ub = (cb >= 'a' && cb <= 'z') ? cb - 32 : cb;
                        if (ca == '-' || cb == '-') mk = ' ';
                        else if (ua == ub) mk = '|';
                        else mk = ((rowpos[ia + p] >> lut[cb]) & 1u) ? ':' : '.';
                    }
                    c0 = ca; c1 = mk; c2 = cb;
                } else if (type == 1) {
                    c0 = '-'; c1 = ' '; c2 = rd[jb + p];
                } else {
                    c0 = amp[ia + p]; c1 = ' '; c2 = '-';
                }
                rows[col + p] = c0;
                rows[stride + col + p] = c1;
                rows[2 * stride + col + p] = c2;
            }
            col += len;
            if (type != 1) ia += len;
            if (type != 2) jb += len;
        }
        nw::lds_fence();
        uint32_t* dst = (uint32_t*)(aln + r * 3 * stride);
        const uint32_t* src = (const uint32_t*)rows;
        const int words = (L + 3) >> 2, sw = (int)(stride >> 2);
        for (int w = lane; w < words; w += 64) {
            dst[w] = src[w];
            dst[sw + w] = src[sw + w];
            dst[2 * sw + w] = src[2 * sw + w];
        }
        nw::lds_fence();
    }
}

// ---------------------------------------------------------------------------
// quant_lanes: process_df_chunk straight from the aligner's traceback runs, one LANE per read.
//
// The row kernels above rebuild three rows per read (3 * aln_len bytes written to HBM and read
// back) and then find the '.' / '-' runs of the rows with a wave per read.  The runs already
// are those features: a Y run is a run of '-' in align_seq (a deletion, CORE:496-502), an X run
// a run of '-' in ref_seq (an insertion, CORE:509-526), and the '.' columns of align_str (the
// substitutions, CORE:486-492) are the non-identical, non-positive pairs of the M runs -- of
// which the record says how many there are: M columns - n_ident (M = La + Lb - aln_len), so an
// M run is scanned (4 columns per step against the amplicon in LDS) only while some are left.
// compute_ref_positions (CORE:2055-2067) of an amplicon made of A C G T is the amplicon index
// of every M / Y column; an insertion's flanks are the columns either side (CORE:520-526, with
// its -1 / -idx at the ends).  Each lane then classifies its read and applies the window and
// frameshift rules exactly as quant_kernel does (same flags, same quirks), and adds its
// positions to the block's vectors once per distinct position (numpy's buffered
// `vec[idx] += 1`): substitution and deletion positions are distinct amplicon bases, insertion
// flanks are deduplicated against them and each other.
//
// Scope: an amplicon of A C G T only, no N rule (amplicon_has_n); everything else of the read
// is handled except a '-' byte in the read (RC-retry input, CORE:1846: it makes a '-' column
// of align_seq inside an M or X run) and more than kQS / kQD / kQI substitutions / deletions /
// insertions: such a read goes to the fallback list, which expand_rows + quant_kernel process
// after this kernel (the same results, by the row path).
//
// Occupancy (round 6): the lists are small (a C2 read has at most one indel and a few substitutions;
// more go to the row path) and each wave first queues the reads of its 256 that need work (60 % of a
// C2 batch are UNMODIFIED on input), so every lane of the main loop holds a read; blocks of 8 waves.
constexpr int kQS = 8, kQD = 2, kQI = 2;    // per-lane list capacities (LDS, [cap][64] per wave)
constexpr int kQSuper = 128;                // reads a wave queues at a time (uint16 queue in LDS)
constexpr int kQStep = 32;                  // M-run columns compared per step (their loads in flight together)
constexpr int kQWaveWords = kQS * 64 / 2 + (kQD + kQI) * 64 * 2 + kQSuper / 2;

struct LArgs {
    const uint32_t* ops;
    const int64_t* ops_off;
    const int32_t* stats;     // nw_stat records (8 ints): aln_len, n_ident, ...
    const uint8_t* reads;
    const int64_t* offsets;
    int64_t bias;
    const uint8_t* amp;       // the amplicon (global; staged into LDS)
    const uint32_t* rowpos;   // per amplicon position: EDNAFULL codes scoring > 0 against it (':' test)
    const uint8_t* lut;       // ascii -> EDNAFULL code
    const uint8_t* pre;
    int64_t n;
    int64_t stride;           // the rows' stride of the row path (aln_len above it: cls -1, as there)
    int4* out;
    uint32_t* partial;        // [gridDim.x][nwords]
    const int32_t* prefix;
    int32_t* fb_list;         // reads this kernel leaves to the row path
    int32_t* fb_count;
    int32_t LEN, H, window, nwords, base_words, amp_words;
    uint32_t flags;
};

__global__ __launch_bounds__(512) void quant_lanes(const LArgs a) {
    extern __shared__ uint32_t smem[];
    const int LEN = a.LEN;
    uint32_t* blk = smem;
    int32_t* incp = (int32_t*)(blk + a.nwords);
    int32_t* exop = incp + (LEN + 1);
    int32_t* splp = exop + (LEN + 1);
    uint8_t* tbl = (uint8_t*)(splp + (LEN + 1));
    uint32_t* amp32 = smem + a.base_words;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    uint16_t* subl = (uint16_t*)(amp32 + a.amp_words + wave * kQWaveWords);   // [kQS][64]
    uint2* dell = (uint2*)(subl + kQS * 64);                                    // [kQD][64]
    uint2* insl = dell + kQD * 64;                                              // [kQI][64]
    uint16_t* queue = (uint16_t*)(insl + kQI * 64);                             // [kQSuper]

    for (int i = threadIdx.x; i < a.nwords; i += blockDim.x) blk[i] = 0;
    const int pref_words = 3 * (LEN + 1) + (LEN + 3) / 4;
    for (int i = threadIdx.x; i < pref_words; i += blockDim.x) incp[i] = a.prefix[i];
    for (int i = threadIdx.x; i < a.amp_words; i += blockDim.x) {
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b)
            if (4 * i + b < LEN) w |= (uint32_t)a.amp[4 * i + b] << (8 * b);
        amp32[i] = w;
    }
    __syncthreads();

    const unsigned flags = a.flags;
    const bool hide = flags & F_HIDE;
    const bool ign_sub = flags & F_IGN_SUB, ign_ins = flags & F_IGN_INS, ign_del = flags & F_IGN_DEL;
    uint32_t* ctr = blk + NV * LEN;
    uint32_t* hin = ctr + 4;
    uint32_t* hfs = hin + a.H;

    const int64_t nsuper = (a.n + kQSuper - 1) / kQSuper;
    const int64_t tw = (int64_t)gridDim.x * wpb;
    for (int64_t sg = (int64_t)blockIdx.x * wpb + wave; sg < nsuper; sg += tw) {
        // queue the reads that need work (not UNMODIFIED, a valid length); the others' results now
        const int64_t r_base = sg * kQSuper;
        int qn = 0;
        for (int h = 0; h < kQSuper / 64; ++h) {
            const int64_t r = r_base + 64 * h + lane;
            const bool valid = r < a.n;
            const unsigned pre = valid ? (unsigned)a.pre[r] : (unsigned)NWQ_PRE_UNMODIFIED;
            const int L = valid ? a.stats[r * 8] : 1;
            const bool skip = pre & NWQ_PRE_UNMODIFIED;
            const bool badlen = L <= 0 || L > a.stride;
            const bool act = valid && !skip && !badlen;
            if (valid && !act) a.out[r] = make_int4((!skip && badlen) ? -1 : 0, 0, 0, 0);
            const unsigned long long m = ballot(act);
            if (act)
                queue[qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                    (uint16_t)(64 * h + lane);
            qn += __popcll(m);
        }
        nw::lds_fence();
        for (int q0 = 0; q0 < qn; q0 += 64) {
            const bool act = q0 + lane < qn;
            const int64_t r = act ? r_base + queue[q0 + lane] : a.n;
            const bool valid = act;
            const unsigned pre = act ? (unsigned)a.pre[r] : (unsigned)NWQ_PRE_UNMODIFIED;
            const int L = act ? a.stats[r * 8] : 1;
            int4 res = make_int4(0, 0, 0, 0);
            bool fb = false, bad = false;
            int nsub = 0, nsubi = 0, nd = 0, ni = 0;
            unsigned subbits = 0;   // 1 exon, 2 splice, 4 exon & include, 8 splice & include
            if (act) {
                const int nid = a.stats[r * 8 + 1];
                const int64_t k0 = a.ops_off[r], k1 = a.ops_off[r + 1];
                const int64_t o0 = a.offsets[r];
                const int Lb = (int)(a.offsets[r + 1] - o0);
                const uint8_t* R = a.reads + (o0 - a.bias);
                int left = LEN + Lb - L - nid;   // non-identical M columns
                fb = left < 0;
                int col = 0, ia = 0, jb = 0, ctype = -1, clen = 0;
                for (int64_t k = k0; k <= k1 && !fb && !bad; ++k) {
                    int t = -2, l = 0;
                    if (k < k1) {
                        const uint32_t op = a.ops[k];
                        t = (int)(op >> 28);
                        l = (int)(op & 0x0fffffffu);
                    }
                    if (t == ctype) {   // consecutive runs of one type: one column run
                        clen += l;
                        continue;
                    }
                    if (ctype == 0) {   // M: the '.' columns among the non-identical ones
                        if (ia + clen > LEN) {
                            bad = true;
                        } else if (left > 0) {
                            // kQStep columns per step: the read's next kQStep / 4 dwords loaded together
                            // (one round trip per kQStep columns instead of per 4), the amplicon's from LDS
                            const uintptr_t ra = (uintptr_t)(R + jb);
                            const uint32_t* rw = (const uint32_t*)(ra & ~(uintptr_t)3);
                            const int rsh = (int)(ra & 3), ash = ia & 3;
                            const int wlast = (rsh + clen) >> 2;   // the last dword a step may read
                            const uint32_t* aw = amp32 + (ia >> 2);
                            uint32_t rlo = rw[0], alo = aw[0];
                            for (int p = 0, q = 0; p < clen && left > 0 && !fb; p += kQStep, q += kQStep / 4) {
                                uint32_t rn[kQStep / 4], an[kQStep / 4];
#pragma unroll
                                for (int i = 0; i < kQStep / 4; ++i) {
                                    rn[i] = q + 1 + i <= wlast ? rw[q + 1 + i] : 0u;
                                    an[i] = aw[q + 1 + i];
                                }
#pragma unroll
                                for (int i = 0; i < kQStep / 4; ++i) {
                                    const int pi = p + 4 * i;
                                    const uint32_t rv = __builtin_amdgcn_alignbyte(rn[i], i ? rn[i - 1] : rlo, rsh);
                                    const uint32_t av = __builtin_amdgcn_alignbyte(an[i], i ? an[i - 1] : alo, ash);
                                    uint32_t x = (pi < clen && !fb) ? rv ^ av : 0u;
                                    if (clen - pi < 4) x &= (1u << (8 * (clen - pi))) - 1u;
                                    while (x) {
                                        const int b = __builtin_ctz(x) >> 3;
                                        x &= ~(255u << (8 * b));
                                        const unsigned cb = (rv >> (8 * b)) & 255u, ca = (av >> (8 * b)) & 255u;
                                        if (cb == '-') {   // a '-' byte of the read: a deletion column of align_seq
                                            fb = true;
                                            break;
                                        }
                                        if ((cb ^ ca) == 0x20u && cb >= 'a' && cb <= 'z') continue;   // '|' (case)
                                        --left;
                                        const int qp = ia + pi + b;
                                        if ((a.rowpos[qp] >> a.lut[cb]) & 1u) continue;   // ':'
                                        if (ign_sub) continue;
                                        if (nsub >= kQS) {
                                            fb = true;
                                            break;
                                        }
                                        subl[nsub * 64 + lane] = (uint16_t)qp;
                                        ++nsub;
                                        const unsigned tb = tbl[qp];
                                        nsubi += tb & T_INC;
                                        subbits |= ((tb & T_EXON) ? 1u : 0u) | ((tb & T_SPL) ? 2u : 0u);
                                        if (tb & T_INC) subbits |= ((tb & T_EXON) ? 4u : 0u) | ((tb & T_SPL) ? 8u : 0u);
                                    }
                                }
                                rlo = rn[kQStep / 4 - 1];
                                alo = an[kQStep / 4 - 1];
                            }
                        }
                        col += clen;
                        ia += clen;
                        jb += clen;
                    } else if (ctype == 2) {   // Y: a deletion (its amplicon positions)
                        if (ia + clen > LEN) {
                            bad = true;
                        } else if (!ign_del) {
                            if (nd >= kQD) {
                                fb = true;
                            } else {
                                const int e = ia + clen;
                                const unsigned f = (incp[e] - incp[ia] > 0 ? R_INC : 0) | (splp[e] - splp[ia] > 0 ? R_SPL : 0);
                                dell[nd * 64 + lane] = make_uint2((unsigned)ia | ((unsigned)clen << 16),
                                                                  f | ((unsigned)(exop[e] - exop[ia]) << 16));
                                ++nd;
                            }
                        }
                        col += clen;
                        ia += clen;
                    } else if (ctype == 1) {   // X: an insertion (its flanking reference positions)
                        for (int p = 0; p < clen && !fb; ++p) fb = R[jb + p] == '-';
                        if (!ign_ins && !fb) {
                            if (ni >= kQI) {
                                fb = true;
                            } else {
                                const int fa = col > 0 ? ia - 1 : -1;
                                const int fbk = col + clen < L ? ia : (ia > 0 ? -ia : -1);
                                unsigned f = 0;   // T_* and R_INC / R_EXON / R_SPL share bit positions
                                if (fa >= 0 && fa < LEN) f |= tbl[fa];
                                if (fbk >= 0 && fbk < LEN) f |= tbl[fbk];
                                insl[ni * 64 + lane] = make_uint2(((unsigned)fa & 0xffffu) | ((unsigned)fbk << 16),
                                                                  (unsigned)clen | (f << 24));
                                ++ni;
                            }
                        }
                        col += clen;
                        jb += clen;
                    } else if (ctype >= 3) {
                        fb = true;
                    }
                    ctype = t;
                    clen = l;
                }
                if (!fb && !bad && (col != L || jb != Lb)) fb = true;
                if (!fb && !bad && ia != LEN) bad = true;
                if (bad) res = make_int4(-1, 0, 0, 0);
            }
            // the reads left to the row path: one atomic per wave
            {
                const unsigned long long fbm = ballot(fb);
                if (fbm) {
                    int base = 0;
                    if (lane == 0) base = atomicAdd(a.fb_count, __popcll(fbm));
                    base = __builtin_amdgcn_readfirstlane(base);
                    if (fb) a.fb_list[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(fbm >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((unsigned)fbm, 0u))] = (int32_t)r;
                }
            }
            if (act && !fb && !bad) {
                // classification (CORE:530-575)
                bool hit = nsubi > 0;
                for (int j = 0; j < nd; ++j) hit |= (dell[j * 64 + lane].y & R_INC) != 0;
                for (int j = 0; j < ni; ++j) hit |= ((insl[j * 64 + lane].y >> 24) & R_INC) != 0;
                const int cls = (pre & NWQ_PRE_HDR) ? 2 : (pre & NWQ_PRE_MIXED) ? 3 : hit ? 1 : 0;
                const bool windowed = cls == 1 && a.window != 0;
                // NHEJ window filter (CORE:611-641): deletion_positions_flat is recomputed only when
                // a deletion survives the filter
                bool anykept = false;
                for (int j = 0; j < nd; ++j) anykept |= !windowed || (dell[j * 64 + lane].y & R_INC);
                const bool post_sel = windowed && anykept;
                int ndel = 0, exdel = 0;
                bool spldel = false;
                for (int j = 0; j < nd; ++j) {
                    uint2 d = dell[j * 64 + lane];
                    const bool kept = !windowed || (d.y & R_INC);
                    const bool post = post_sel ? kept : true;
                    d.y |= (kept ? R_KEPT : 0) | (post ? R_POST : 0);
                    dell[j * 64 + lane] = d;
                    ndel += kept ? (int)(d.x >> 16) : 0;
                    exdel += post ? (int)(d.y >> 16) : 0;
                    spldel |= post && (d.y & R_SPL);
                }
                int nins = 0, insex_len = 0;
                bool insex = false, insspl = false;
                for (int j = 0; j < ni; ++j) {
                    const uint2 e = insl[j * 64 + lane];
                    const int fa = (int)(short)(e.x & 0xffffu), fbk = (int)(short)(e.x >> 16);
                    const int sz = (int)(e.y & 0xffffffu);
                    const unsigned f = e.y >> 24;
                    const bool kept = !windowed || (f & R_INC);
                    insspl |= (f & R_SPL) != 0;
                    if (kept) {
                        nins += sz;
                        if (f & R_EXON) {
                            insex = true;
                            insex_len += sz;
                        }
                        if (cls != 0) {
                            const int wa = fa < 0 ? fa + LEN : fa, wb = fbk < 0 ? fbk + LEN : fbk;
                            atomicAdd(blk + V_AVG_INS * LEN + wa, (unsigned)sz);
                            if (wb != wa) atomicAdd(blk + V_AVG_INS * LEN + wb, (unsigned)sz);
                        }
                    }
                }
                const int n_mut = windowed ? nsubi : nsub;
                bool noncoding = false;
                if ((flags & F_FRAMESHIFT) && cls != 0) {   // CORE:653-725
                    const bool sub_exon = windowed ? (subbits & 4u) : (subbits & 1u);
                    const bool sub_spl = windowed ? (subbits & 8u) : (subbits & 2u);
                    const int eff = insex_len - exdel;
                    const bool exon_mod = insex || exdel > 0 || sub_exon;
                    const bool has_lens = insex || exdel > 0;
                    if (sub_spl || spldel || insspl) atomicAdd(ctr + C_SPLICE, 1u);
                    if (exon_mod) {
                        if (!has_lens) {
                            atomicAdd(ctr + C_NONFS, 1u);
                            atomicAdd(hin + LEN, 1u);
                        } else if (eff % 3 == 0) {
                            atomicAdd(ctr + C_NONFS, 1u);
                            atomicAdd(hin + LEN + eff, 1u);
                        } else {
                            atomicAdd(ctr + C_FS, 1u);
                            atomicAdd(hfs + LEN + eff, 1u);
                        }
                    } else {
                        atomicAdd(ctr + C_NONMOD, 1u);
                    }
                    noncoding = !exon_mod;
                }
                res = cls ? make_int4(cls, n_mut, nins, ndel) : make_int4(0, 0, 0, 0);

                // the read's vector increments, once per distinct position
                auto is_flank = [&](int p) {
                    for (int j = 0; j < ni; ++j) {
                        const unsigned x = insl[j * 64 + lane].x;
                        const int fa = (int)(short)(x & 0xffffu), fbk = (int)(short)(x >> 16);
                        if ((fa < 0 ? fa + LEN : fa) == p || (fbk < 0 ? fbk + LEN : fbk) == p) return true;
                    }
                    return false;
                };
                auto incr = [&](int p, unsigned sub, unsigned del, unsigned ins, unsigned sub_post, unsigned del_post,
                                unsigned dsz, bool kept) {
                    uint32_t* h = blk + p;
                    if (cls == 3) {
                        vadd(h, V_MUT_MIX, LEN, sub); vadd(h, V_DEL_MIX, LEN, del); vadd(h, V_INS_MIX, LEN, ins);
                    } else if (cls == 2) {
                        vadd(h, V_MUT_HDR, LEN, sub); vadd(h, V_DEL_HDR, LEN, del); vadd(h, V_INS_HDR, LEN, ins);
                    } else if (cls == 1) {
                        vadd(h, V_MUT, LEN, hide ? sub_post : sub);
                        vadd(h, V_DEL, LEN, hide ? del_post : del);
                        vadd(h, V_INS, LEN, ins);
                    }
                    vadd(h, V_ANY, LEN, 1u);
                    if (noncoding) {
                        vadd(h, V_MUT_NC, LEN, sub_post); vadd(h, V_DEL_NC, LEN, del_post); vadd(h, V_INS_NC, LEN, ins);
                    }
                    if (cls != 0 && del && kept) vadd(h, V_AVG_DEL, LEN, dsz);
                };
                for (int j = 0; j < nsub; ++j) {
                    const int p = subl[j * 64 + lane];
                    const unsigned sp = (!windowed || (tbl[p] & T_INC)) ? 1u : 0u;
                    incr(p, 1u, 0u, is_flank(p) ? 1u : 0u, sp, 0u, 0u, false);
                }
                for (int j = 0; j < nd; ++j) {
                    const uint2 d = dell[j * 64 + lane];
                    const int s = (int)(d.x & 0xffffu), sz = (int)(d.x >> 16);
                    const unsigned dp = (d.y & R_POST) ? 1u : 0u;
                    const bool kept = d.y & R_KEPT;
                    for (int p = s; p < s + sz; ++p) incr(p, 0u, 1u, (ni && is_flank(p)) ? 1u : 0u, 0u, dp, (unsigned)sz, kept);
                }
                for (int j = 0; j < ni; ++j) {
                    const unsigned x = insl[j * 64 + lane].x;
                    const int fa = (int)(short)(x & 0xffffu), fbk = (int)(short)(x >> 16);
                    const int w2[2] = {fa < 0 ? fa + LEN : fa, fbk < 0 ? fbk + LEN : fbk};
                    for (int h = 0; h < 2; ++h) {
                        const int w = w2[h];
                        if (h == 1 && w == w2[0]) continue;
                        bool seen = false;
                        for (int jj = 0; jj < j && !seen; ++jj) {
                            const unsigned xx = insl[jj * 64 + lane].x;
                            const int ga = (int)(short)(xx & 0xffffu), gb = (int)(short)(xx >> 16);
                            seen = (ga < 0 ? ga + LEN : ga) == w || (gb < 0 ? gb + LEN : gb) == w;
                        }
                        for (int q = 0; q < nsub && !seen; ++q) seen = subl[q * 64 + lane] == w;
                        for (int q = 0; q < nd && !seen; ++q) {
                            const unsigned dx = dell[q * 64 + lane].x;
                            seen = w >= (int)(dx & 0xffffu) && w < (int)(dx & 0xffffu) + (int)(dx >> 16);
                        }
                        if (!seen) incr(w, 0u, 0u, 1u, 0u, 0u, 0u, false);
                    }
                }
            }
            if (valid && !fb) a.out[r] = res;
        }
        nw::lds_fence();   // every lane's queue reads before the next super-group's writes
    }

    __syncthreads();
    uint32_t* dst = a.partial + (int64_t)blockIdx.x * a.nwords;
    for (int i = threadIdx.x; i < a.nwords; i += blockDim.x) dst[i] = blk[i];
}

__global__ void quant_reduce(const uint32_t* __restrict__ partial, int nblocks, int nwords, int slice,
                             unsigned long long* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nwords) return;
    const int b0 = blockIdx.y * slice, b1 = min(nblocks, b0 + slice);
    unsigned long long s = 0;
    for (int b = b0; b < b1; ++b) s += partial[(int64_t)b * nwords + i];
    if (s) atomicAdd(out + i, s);
}


}  // namespace nwq

// ------------------------------------------------------------------ host side

namespace {

template <class T>
struct QBuf {
    T* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

constexpr int kMaxLds = 160 * 1024;

}  // namespace

struct nwq_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    bool have_params = false;
    int32_t LEN = 0;
    uint32_t flags = 0;
    int32_t window = 0;
    int64_t lane_fallbacks = -1;     // the last nwq_run_device_ops' quant_lanes fallback count
    std::vector<int32_t> prefix;     // host copy of QArgs::prefix
    QBuf<int32_t> d_prefix;
    QBuf<uint32_t> d_partial;
    QBuf<int64_t> d_totals;
    QBuf<uint8_t> d_aln, d_pre;
    QBuf<int32_t> d_len;
    QBuf<nwq_read> d_out;
    // nwq_run_device_ops: the amplicon, its positive-code masks, ascii -> EDNAFULL code
    QBuf<uint8_t> d_amp, d_lut;
    QBuf<uint32_t> d_rowpos;
    std::string amp_key;
    QBuf<int32_t> d_fb;      // quant_lanes' fallback list [n] + its count
    bool rows_only = false;  // CRISPR_NWQ_ROWS=1: every read through the rows (A/B, tests)
    // page-locked landing space of the call's results (the totals, the fallback count): copied back on
    // the stream before its one synchronisation, no pageable staging or second round trip
    int64_t* h_totals = nullptr;
    int64_t h_totals_cap = 0;
    int32_t* h_nfb = nullptr;
    // blocks per CU of (kernel, block size, LDS) -- the occupancy query once per shape, not per call
    struct Occ { const void* f; int threads, lds, per_cu; };
    Occ occ[8] = {};
    int n_occ = 0;
};

namespace {

int occupancy(nwq_ctx* c, const void* f, int threads, int lds, int* per_cu) {
    for (int i = 0; i < c->n_occ; ++i)
        if (c->occ[i].f == f && c->occ[i].threads == threads && c->occ[i].lds == lds) {
            *per_cu = c->occ[i].per_cu;
            return 0;
        }
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, threads, lds);
    if (e != hipSuccess) return (int)e;
    if (c->n_occ < 8) c->occ[c->n_occ++] = nwq_ctx::Occ{f, threads, lds, *per_cu};
    return 0;
}

int qfail(nwq_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define QHIP(c, expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return qfail((c), NW_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

int64_t hist_size(int32_t LEN, int64_t stride) { return (int64_t)LEN + stride + 1; }
int64_t words_for(int32_t LEN, int64_t stride) { return (int64_t)nwq::NV * LEN + 4 + 2 * hist_size(LEN, stride); }

struct QGeom {
    int wpb, grid, lds, run_cap, wave_words, base_words, nwords;
};

int geometry(nwq_ctx* c, int64_t stride, int64_t n, QGeom* g) {
    const int LEN = c->LEN;
    g->nwords = (int)words_for(LEN, stride);
    g->run_cap = (int)((stride + 1) / 2 + 1);
    const int pref_words = 3 * (LEN + 1) + (LEN + 3) / 4;
    g->base_words = (g->nwords + pref_words + 1) & ~1;
    g->wave_words = ((LEN + 1) & ~1) + 4 * g->run_cap;
    g->wpb = 0;
    for (int w : {8, 4, 2, 1}) {
        const int lds = 4 * (g->base_words + w * g->wave_words);
        // at least two blocks per CU unless even a one-wave block needs more
        if (lds <= kMaxLds / 2 || (w == 1 && lds <= kMaxLds)) {
            g->wpb = w;
            g->lds = lds;
            break;
        }
    }
    if (!g->wpb)
        return qfail(c, NW_E_UNSUPPORTED, "quantification state for amplicon length %d / stride %lld exceeds LDS",
                     LEN, (long long)stride);
    int per_cu = 0;
    QHIP(c, (hipError_t)occupancy(c, (const void*)nwq::quant_kernel, 64 * g->wpb, g->lds, &per_cu));
    per_cu = std::max(per_cu, 1);
    const int64_t need = (n + g->wpb - 1) / g->wpb;
    g->grid = (int)std::max<int64_t>(1, std::min<int64_t>(need, (int64_t)c->num_cus * per_cu));
    return NW_OK;
}

// The row kernel (quant_kernel) over reads [0, n), or over a device work list (list /
// list_count: quant_lanes' fallback reads, `slabs0` block slabs of that kernel already at the
// start of d_partial), then the slabs' sum into the totals.
int run_impl(nwq_ctx* c, uint8_t* d_aln, int64_t stride, const int32_t* d_len, int64_t len_stride,
             const uint8_t* d_pre, int64_t n, nwq_read* d_out, int64_t* totals, float* kernel_ms,
             bool started = false, const int32_t* list = nullptr, const int32_t* list_count = nullptr,
             int slabs0 = 0, int32_t* nfb = nullptr) {
    if (!c->have_params) return qfail(c, NW_E_STATE, "nwq_set_params not called");
    if (stride <= 0 || (stride & 3) || stride >= 32768)
        return qfail(c, NW_E_INVALID, "stride %lld must be a positive multiple of 4 below 32768", (long long)stride);
    if (n < 0) return qfail(c, NW_E_INVALID, "negative read count");
    QGeom g;
    int rc = geometry(c, stride, n, &g);
    if (rc) return rc;
    if (list) g.grid = std::min(g.grid, c->num_cus);   // a short list (usually empty): a small grid
    QHIP(c, c->d_partial.reserve((size_t)(slabs0 + g.grid) * g.nwords));
    QHIP(c, c->d_totals.reserve((size_t)g.nwords));
    nwq::QArgs a;
    a.aln = d_aln;
    a.stride = stride;
    a.len = d_len;
    a.len_stride = len_stride;
    a.pre = d_pre;
    a.n = n;
    a.out = reinterpret_cast<int4*>(d_out);
    a.partial = c->d_partial.p + (size_t)slabs0 * g.nwords;
    a.prefix = c->d_prefix.p;
    a.list = list;
    a.list_count = list_count;
    a.LEN = c->LEN;
    a.H = (int)hist_size(c->LEN, stride);
    a.run_cap = g.run_cap;
    a.window = c->window;
    a.nwords = g.nwords;
    a.wave_words = g.wave_words;
    a.base_words = g.base_words;
    a.flags = c->flags;
    if (!started) QHIP(c, hipEventRecord(c->ev0, c->stream));   // (the row expansion records it first)
    hipLaunchKernelGGL(nwq::quant_kernel, dim3(g.grid), dim3(64 * g.wpb), g.lds, c->stream, a);
    QHIP(c, hipGetLastError());
    const int nslabs = slabs0 + g.grid;
    const int slices = std::min(nslabs, 32), slice = (nslabs + slices - 1) / slices;
    QHIP(c, hipMemsetAsync(c->d_totals.p, 0, sizeof(int64_t) * (size_t)g.nwords, c->stream));
    hipLaunchKernelGGL(nwq::quant_reduce, dim3((g.nwords + 255) / 256, slices), dim3(256), 0, c->stream,
                       c->d_partial.p, nslabs, g.nwords, slice, reinterpret_cast<unsigned long long*>(c->d_totals.p));
    QHIP(c, hipGetLastError());
    QHIP(c, hipEventRecord(c->ev1, c->stream));
    if (c->h_totals_cap < g.nwords) {
        if (c->h_totals) (void)hipHostFree(c->h_totals);
        c->h_totals = nullptr;
        c->h_totals_cap = 0;
        QHIP(c, hipHostMalloc((void**)&c->h_totals, sizeof(int64_t) * (size_t)g.nwords, hipHostMallocDefault));
        c->h_totals_cap = g.nwords;
    }
    QHIP(c, hipMemcpyAsync(c->h_totals, c->d_totals.p, sizeof(int64_t) * (size_t)g.nwords, hipMemcpyDeviceToHost,
                           c->stream));
    if (nfb && list_count) QHIP(c, hipMemcpyAsync(c->h_nfb, list_count, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    QHIP(c, hipStreamSynchronize(c->stream));
    std::memcpy(totals, c->h_totals, sizeof(int64_t) * (size_t)g.nwords);
    if (nfb && list_count) *nfb = *c->h_nfb;
    if (kernel_ms) QHIP(c, hipEventElapsedTime(kernel_ms, c->ev0, c->ev1));
    return NW_OK;
}

}  // namespace

extern "C" {

int64_t nwq_lane_fallbacks(const nwq_ctx* c) { return c ? c->lane_fallbacks : -1; }

int nwq_create(int device, nwq_ctx** out) {
    if (!out) return NW_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NW_E_HIP;
    nwq_ctx* c = new nwq_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipHostMalloc((void**)&c->h_nfb, sizeof(int32_t), hipHostMallocDefault) != hipSuccess) {
        nwq_destroy(c);
        return NW_E_HIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    if (const char* e = std::getenv("CRISPR_NWQ_ROWS")) c->rows_only = std::strcmp(e, "1") == 0;
    *out = c;
    return NW_OK;
}

void nwq_destroy(nwq_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    c->d_prefix.release();
    c->d_partial.release();
    c->d_totals.release();
    c->d_aln.release();
    c->d_pre.release();
    c->d_len.release();
    c->d_out.release();
    c->d_amp.release();
    c->d_lut.release();
    c->d_rowpos.release();
    c->d_fb.release();
    if (c->h_totals) (void)hipHostFree(c->h_totals);
    if (c->h_nfb) (void)hipHostFree(c->h_nfb);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* nwq_last_error(const nwq_ctx* c) { return c ? c->err.c_str() : "null context"; }

int nwq_set_params(nwq_ctx* c, const nwq_params* p) {
    if (!c || !p) return NW_E_INVALID;
    const int LEN = p->len_amplicon;
    if (LEN <= 0 || LEN >= 32768) return qfail(c, NW_E_INVALID, "len_amplicon %d out of range (1..32767)", LEN);
    if (!p->include_mask) return qfail(c, NW_E_INVALID, "include_mask is required");
    if (hipSetDevice(c->device) != hipSuccess) return qfail(c, NW_E_HIP, "hipSetDevice failed");
    const int pref_words = 3 * (LEN + 1) + (LEN + 3) / 4;
    c->prefix.assign((size_t)pref_words, 0);
    int32_t* inc = c->prefix.data();
    int32_t* exo = inc + (LEN + 1);
    int32_t* spl = exo + (LEN + 1);
    uint8_t* tbl = reinterpret_cast<uint8_t*>(spl + (LEN + 1));
    for (int i = 0; i < LEN; ++i) {
        const bool bi = p->include_mask[i] != 0;
        const bool be = p->exon_mask && p->exon_mask[i];
        const bool bs = p->exon_mask && p->splicing_mask && p->splicing_mask[i];
        tbl[i] = (uint8_t)((bi ? nwq::T_INC : 0) | (be ? nwq::T_EXON : 0) | (bs ? nwq::T_SPL : 0));
        inc[i + 1] = inc[i] + bi;
        exo[i + 1] = exo[i] + be;
        spl[i + 1] = spl[i] + bs;
    }
    QHIP(c, c->d_prefix.reserve((size_t)pref_words));
    QHIP(c, hipMemcpy(c->d_prefix.p, c->prefix.data(), sizeof(int32_t) * (size_t)pref_words, hipMemcpyHostToDevice));
    c->LEN = LEN;
    c->window = p->window_around_sgrna;
    c->flags = (p->ignore_substitutions ? nwq::F_IGN_SUB : 0) | (p->ignore_insertions ? nwq::F_IGN_INS : 0) |
               (p->ignore_deletions ? nwq::F_IGN_DEL : 0) | (p->hide_mutations_outside_window_nhej ? nwq::F_HIDE : 0) |
               (p->exon_mask ? nwq::F_FRAMESHIFT : 0) | (p->amplicon_has_n ? nwq::F_NFIX : 0);
    c->have_params = true;
    return NW_OK;
}

int64_t nwq_totals_words(const nwq_ctx* c, int64_t stride) {
    return (c && c->have_params) ? words_for(c->LEN, stride) : 0;
}

int nwq_run(nwq_ctx* c, uint8_t* aln, int64_t stride, const int32_t* aln_len, const uint8_t* pre, int64_t n,
            nwq_read* out, int64_t* totals, float* kernel_ms) {
    if (!c) return NW_E_INVALID;
    if (n > 0 && (!aln || !aln_len || !pre || !out)) return qfail(c, NW_E_INVALID, "null buffer");
    if (!totals) return qfail(c, NW_E_INVALID, "null totals");
    QHIP(c, hipSetDevice(c->device));
    const size_t nn = (size_t)std::max<int64_t>(n, 1);
    QHIP(c, c->d_aln.reserve(nn * 3 * (size_t)stride));
    QHIP(c, c->d_len.reserve(nn));
    QHIP(c, c->d_pre.reserve(nn));
    QHIP(c, c->d_out.reserve(nn));
    if (n > 0) {
        QHIP(c, hipMemcpyAsync(c->d_aln.p, aln, (size_t)n * 3 * stride, hipMemcpyHostToDevice, c->stream));
        QHIP(c, hipMemcpyAsync(c->d_len.p, aln_len, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, c->stream));
        QHIP(c, hipMemcpyAsync(c->d_pre.p, pre, (size_t)n, hipMemcpyHostToDevice, c->stream));
    }
    int rc = run_impl(c, c->d_aln.p, stride, c->d_len.p, 1, c->d_pre.p, n, c->d_out.p, totals, kernel_ms);
    if (rc) return rc;
    if (n > 0) {
        QHIP(c, hipMemcpy(out, c->d_out.p, sizeof(nwq_read) * (size_t)n, hipMemcpyDeviceToHost));
        if (c->flags & nwq::F_NFIX)
            QHIP(c, hipMemcpy2D(aln + stride, (size_t)(3 * stride), c->d_aln.p + stride, (size_t)(3 * stride),
                                (size_t)stride, (size_t)n, hipMemcpyDeviceToHost));
    }
    return NW_OK;
}

int nwq_run_device(nwq_ctx* c, uint8_t* d_aln, int64_t stride, const int32_t* d_aln_len, int64_t len_stride,
                   const uint8_t* d_pre, int64_t n, nwq_read* d_out, int64_t* totals, float* kernel_ms) {
    if (!c) return NW_E_INVALID;
    if (n > 0 && (!d_aln || !d_aln_len || !d_pre || !d_out)) return qfail(c, NW_E_INVALID, "null buffer");
    if (!totals) return qfail(c, NW_E_INVALID, "null totals");
    if (len_stride <= 0) return qfail(c, NW_E_INVALID, "len_stride must be positive");
    QHIP(c, hipSetDevice(c->device));
    return run_impl(c, d_aln, stride, d_aln_len, len_stride, d_pre, n, d_out, totals, kernel_ms);
}

int nwq_run_device_ops(nwq_ctx* c, const char* amplicon, int32_t amplicon_len, const uint32_t* d_ops,
                       const int64_t* d_ops_off, const void* d_stats, const uint8_t* d_reads, const int64_t* d_offsets,
                       int64_t reads_bias, int64_t stride, const uint8_t* d_pre, int64_t n, nwq_read* d_out,
                       int64_t* totals, float* kernel_ms) {
    if (!c) return NW_E_INVALID;
    if (!c->have_params) return qfail(c, NW_E_STATE, "nwq_set_params not called");
    if (!amplicon || amplicon_len != c->LEN)
        return qfail(c, NW_E_INVALID, "amplicon of %d bases for len_amplicon %d", amplicon_len, c->LEN);
    if (n > 0 && (!d_ops || !d_ops_off || !d_stats || !d_reads || !d_offsets || !d_pre || !d_out))
        return qfail(c, NW_E_INVALID, "null buffer");
    if (!totals) return qfail(c, NW_E_INVALID, "null totals");
    if (stride <= 0 || (stride & 3) || stride >= 32768)
        return qfail(c, NW_E_INVALID, "stride %lld must be a positive multiple of 4 below 32768", (long long)stride);
    QHIP(c, hipSetDevice(c->device));
    const std::string key(amplicon, amplicon + amplicon_len);
    if (key != c->amp_key) {   // the amplicon's tables (the markup's ':' test), once per amplicon
        std::vector<uint32_t> rowpos((size_t)amplicon_len);
        std::vector<uint8_t> lut(256);
        for (int b = 0; b < 256; ++b) lut[(size_t)b] = nw::code_of((unsigned char)b);
        for (int i = 0; i < amplicon_len; ++i) {
            const int ca = nw::code_of((unsigned char)amplicon[i]);
            uint32_t m = 0;
            for (int code = 0; code < 16; ++code)
                if (ca < 16 && nw::kEdna[ca][code] > 0) m |= 1u << code;
            rowpos[(size_t)i] = m;
        }
        QHIP(c, c->d_amp.reserve((size_t)amplicon_len + 16));
        QHIP(c, c->d_rowpos.reserve((size_t)amplicon_len));
        QHIP(c, c->d_lut.reserve(256));
        QHIP(c, hipMemcpy(c->d_amp.p, amplicon, (size_t)amplicon_len, hipMemcpyHostToDevice));
        QHIP(c, hipMemcpy(c->d_rowpos.p, rowpos.data(), 4 * rowpos.size(), hipMemcpyHostToDevice));
        QHIP(c, hipMemcpy(c->d_lut.p, lut.data(), 256, hipMemcpyHostToDevice));
        c->amp_key = key;
    }
    const size_t nn = (size_t)std::max<int64_t>(n, 1);
    QHIP(c, c->d_aln.reserve(nn * 3 * (size_t)stride));
    // the lane path (quant_lanes: features straight from the runs) for an amplicon of A C G T
    // without the N rule, when its LDS fits; its fallback reads (and every read otherwise) go
    // through the rows rebuilt on the device
    bool acgt = true;
    for (int i = 0; i < amplicon_len && acgt; ++i)
        acgt = amplicon[i] == 'A' || amplicon[i] == 'C' || amplicon[i] == 'G' || amplicon[i] == 'T';
    const int LEN = c->LEN;
    const int nwords = (int)words_for(LEN, stride);
    const int pref_words = 3 * (LEN + 1) + (LEN + 3) / 4;
    const int base_words = nwords + pref_words;
    const int amp_words = (LEN + 3) / 4 + 2;
    int lane_wpb = 8;
    while (lane_wpb > 1 && 4 * (base_words + amp_words + lane_wpb * nwq::kQWaveWords) > kMaxLds / 2) lane_wpb >>= 1;
    const int lane_lds = 4 * (base_words + amp_words + lane_wpb * nwq::kQWaveWords);
    const bool lanes = acgt && !(c->flags & nwq::F_NFIX) && lane_lds <= kMaxLds && n > 0 && !c->rows_only;
    QHIP(c, hipEventRecord(c->ev0, c->stream));   // kernel_ms covers the expansion too
    c->lane_fallbacks = -1;
    if (lanes) {
        int per_cu = 0;
        QHIP(c, (hipError_t)occupancy(c, (const void*)nwq::quant_lanes, 64 * lane_wpb, lane_lds, &per_cu));
        per_cu = std::max(per_cu, 1);
        const int64_t groups = (n + nwq::kQSuper - 1) / nwq::kQSuper;   // a wave's super-groups
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((groups + lane_wpb - 1) / lane_wpb,
                                                                     (int64_t)c->num_cus * per_cu));
        QHIP(c, c->d_fb.reserve(nn + 1));
        // every slab up front: the row kernel's list grid is at most num_cus (run_impl), and a
        // reserve there would move the slabs this kernel is about to write
        QHIP(c, c->d_partial.reserve((size_t)(grid + c->num_cus) * nwords));
        QHIP(c, hipMemsetAsync(c->d_fb.p + nn, 0, sizeof(int32_t), c->stream));
        nwq::LArgs la;
        la.ops = d_ops;
        la.ops_off = d_ops_off;
        la.stats = (const int32_t*)d_stats;
        la.reads = d_reads;
        la.offsets = d_offsets;
        la.bias = reads_bias;
        la.amp = c->d_amp.p;
        la.rowpos = c->d_rowpos.p;
        la.lut = c->d_lut.p;
        la.pre = d_pre;
        la.n = n;
        la.stride = stride;
        la.out = reinterpret_cast<int4*>(d_out);
        la.partial = c->d_partial.p;
        la.prefix = c->d_prefix.p;
        la.fb_list = c->d_fb.p;
        la.fb_count = c->d_fb.p + nn;
        la.LEN = LEN;
        la.H = (int)hist_size(LEN, stride);
        la.window = c->window;
        la.nwords = nwords;
        la.base_words = base_words;
        la.amp_words = amp_words;
        la.flags = c->flags;
        hipLaunchKernelGGL(nwq::quant_lanes, dim3(grid), dim3(64 * lane_wpb), lane_lds, c->stream, la);
        QHIP(c, hipGetLastError());
        // the fallback reads: their rows, then the row kernel over the list
        int wpb = 4;
        while (wpb > 1 && (int64_t)wpb * 3 * stride > 64 * 1024) wpb >>= 1;
        const int lds = (int)(wpb * 3 * stride);
        if (lds > kMaxLds) return qfail(c, NW_E_UNSUPPORTED, "stride %lld too long for the row expansion", (long long)stride);
        hipLaunchKernelGGL(nwq::expand_rows, dim3(c->num_cus), dim3(64 * wpb), lds, c->stream, d_ops, d_ops_off,
                           (const int32_t*)d_stats, d_reads, d_offsets, reads_bias, c->d_amp.p, c->d_rowpos.p,
                           c->d_lut.p, amplicon_len, d_pre, 0, n, c->d_aln.p, stride, c->d_fb.p, c->d_fb.p + nn);
        QHIP(c, hipGetLastError());
        int32_t nfb = -1;
        const int rc = run_impl(c, c->d_aln.p, stride, (const int32_t*)d_stats, 8, d_pre, n, d_out, totals, kernel_ms,
                                true, c->d_fb.p, c->d_fb.p + nn, grid, &nfb);
        c->lane_fallbacks = rc == NW_OK ? nfb : -1;
        return rc;
    }
    if (n > 0) {
        int wpb = 4;
        while (wpb > 1 && (int64_t)wpb * 3 * stride > 64 * 1024) wpb >>= 1;
        const int lds = (int)(wpb * 3 * stride);
        if (lds > kMaxLds) return qfail(c, NW_E_UNSUPPORTED, "stride %lld too long for the row expansion", (long long)stride);
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + wpb - 1) / wpb, (int64_t)c->num_cus * 16));
        hipLaunchKernelGGL(nwq::expand_rows, dim3(grid), dim3(64 * wpb), lds, c->stream, d_ops, d_ops_off,
                           (const int32_t*)d_stats, d_reads, d_offsets, reads_bias, c->d_amp.p, c->d_rowpos.p,
                           c->d_lut.p, amplicon_len, d_pre, (int)((c->flags & nwq::F_NFIX) != 0), n, c->d_aln.p,
                           stride, nullptr, nullptr);
        QHIP(c, hipGetLastError());
    }
    // the records' aln_len, 8 ints apart (nw_stat)
    return run_impl(c, c->d_aln.p, stride, (const int32_t*)d_stats, 8, d_pre, n, d_out, totals, kernel_ms, true);
}

}  // extern "C"
