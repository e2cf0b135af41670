// estep_df.hip — the value pass of the split E-step as a dataflow over loci.
//
// estep_values (estep_split.hip) replays each locus's structure record in two
// phases with a block barrier after each: every state's constructor and the
// appends that still fit (phase A, a thread per state), then the adds that
// overflow S as chains of selections on lane segments (phase B).  A locus
// therefore ends on its longest chain while the other segments idle (cfg 3's
// E1: 6.8 selection steps per locus on the critical path against 4.7 of work
// per segment; its E2: 11 steps, most segments idle).  A state's list only
// depends on its predecessors' final lists (HaploPair.cpp:35-89), so here the
// block's waves run different loci at once:
//
//   A (waves 0..NA-1) walk the loci in order, each over a fixed share of
//     every locus's states (blocks of 64 of the chain list and of the state
//     range, block k to wave k % NA).  A lane takes a state of the current
//     locus — the chains first, longest first (the record's chain list), then
//     the other states — and, once every predecessor it reads is final (one
//     bit per state of the previous locus), builds the state's list exactly as
//     phase A does: the ordered forward sum, the extension constructor and the
//     appends that fit.  A list that is complete is final at once; a chain's
//     state goes to the chain queue.
//   B (waves NA..NW-1) cut into segments of S lanes (two links per lane) or 2S
//     lanes; a segment takes the next chain from the queue, whatever its locus,
//     and runs its adds with the libstdc++-exact segmented selection
//     (coop_select.hpp), then marks the state final.
//
// Locus j's frontier lives in ring slot j % R (R >= 3).  The first A wave to
// reach locus j opens it (trace record, flags, then the slot published) once
// locus j-R+1 — the last reader of the slot's previous occupant, locus j-R —
// is complete; A runs up to R-2 loci ahead of the oldest open chain.  Every
// list is built by the same operations in the same order as in
// estep_values, so the frontiers, the trace store and the results are
// identical; only the interleaving across states changes.
//
// Queue: a ring of `qcap` words in LDS.  A waves take tickets for their
// entries and B segments tickets to serve (two LDS counters).  The entry of
// ticket t goes to slot t % qcap once the slot holds the empty mark of lap
// t / qcap, which the taker of ticket t - qcap leaves; entries carry their lap
// too, so a segment never takes an entry of another lap and a producer never
// overtakes an earlier lap's.  After the last locus (or an abort) the last A
// wave queues one END entry per segment, so every ticket taken is served.
#include "hmc_internal.hpp"
#include "select.hpp"
#include "coop_select.hpp"
#include "estep_common.hpp"
#include "value_front.hpp"

#ifdef HMC_VARIANTS  // (measured slower than estep_values: the variants library only)
namespace hmc {

namespace {

constexpr int DF_RMAX = 4;
constexpr uint32_t QE_VALID = 1u << 31, QE_END = 1u << 30;
constexpr int QE_LAP = 24;   // bits 24..29: ticket lap
constexpr int QE_SLOT = 21;  // bits 21..23: ring slot; 0..20 state
// Watchdog: a wait that polls this often without progress (~10^8 cycles, far
// beyond any chain) means a broken invariant; the block then stops the
// individual with EST_DF_STALL instead of spinning forever.
constexpr int DF_SPIN_MAX = 1 << 22;
constexpr int DF_STALL = 2;  // DfShared::abort value

struct DfRing {
  unsigned long long rec;  // word offset of the locus's structure record
  unsigned long long tr;   // word offset of its trace record
  int F;
  int done;   // states whose lists are final
  int locus;  // the locus in the slot, published once the slot is open
  int pad;
};

struct DfShared {
  DfRing ring[DF_RMAX];
  unsigned long long tcur;  // next trace word of the individual (the opener of each locus)
  int q_head;   // tickets taken by the B segments
  int q_tail;   // tickets queued by the A waves
  int opening;  // the last locus an A wave has claimed to open
  int a_fin;    // A waves done with the individual
  int abort;    // A stopped the individual (underflow, trace store full)
  int status;   // the individual's status for the final selection
  int q;        // next individual (block broadcast)
  int stall_at, stall_val;  // watchdog diagnostics: site << 24 | wave << 16 | locus, and a value of the site
};

// What a B segment needs to start a chain, written by the A lane that queued
// it (it has all of it in registers): one LDS read instead of a round of
// record loads.  Indexed like the queue.
struct DfChain {
  double tpv;       // m_transition_prob of the state
  uint32_t r, re;   // next add and the end of the state's contributions
  uint32_t k0;      // list length after the appends | differ << 31
  uint32_t wc, wn;  // contribution words of adds r and r + 1
  uint32_t pad;
};

struct DfPlan {
  int o_lpos, o_rpos, o_junk, o_slik, o_smeta, o_sh, o_queue, o_desc, o_ascr, o_flags, o_front;
  int front_stride, flag_words, bytes;
  int R, qcap, qlog, G, sws;  // ring slots, queue slots (2^qlog), segments per B wave, selection slots per B wave
  int na;                     // A waves
};

__host__ __device__ inline int df_slots(int S, bool pair) {
  return pair ? (WAVE / S + 1) * 2 * S : (2 * S > WAVE ? 2 * S : WAVE);
}

// na / nb: A / B waves; fc: LDS states per ring slot; fcap: states per slot
// (HBM tier size, and the flag bits)
__host__ __device__ inline DfPlan df_plan(int S, int fc, int na, int nb, bool pair, int R, int qcap, int fcap) {
  DfPlan p;
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += (bytes + 15) & ~15; return r; };
  const int sl = df_slots(S, pair), pos = pair ? sl : WAVE;
  p.o_lpos = take(nb * pos * 4);
  p.o_rpos = take(nb * pos * 4);
  p.o_junk = take(nb * (pair ? 4 : 2) * WAVE * 4);
  p.o_slik = take(nb * sl * 8);
  p.o_smeta = take(nb * sl * 4);
  p.o_sh = take((int)sizeof(DfShared));
  p.o_queue = take(qcap * 4);
  p.o_desc = take(qcap * (int)sizeof(DfChain));
  p.o_ascr = take(na * WAVE * 4);
  p.flag_words = (fcap + 31) / 32;
  p.o_flags = take(R * p.flag_words * 4);
  p.front_stride = (fc * (24 + 8 * S) + 15) & ~15;
  p.o_front = take(R * p.front_stride);
  p.bytes = o;
  p.R = R;
  p.qcap = qcap;
  p.qlog = 0;
  while ((1 << p.qlog) < qcap) ++p.qlog;
  p.G = pair ? WAVE / S : WAVE / (2 * S);
  p.sws = sl;
  p.na = na;
  return p;
}

// A ring slot's frontier: the value pass's compact frontier (value_front.hpp,
// VFront): [0, fc) in LDS, the rest in HBM.
__host__ __device__ inline size_t df_front_bytes(int fcap, int S) { return k2_front_bytes(fcap, S); }

__device__ inline int ld_vol(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ inline uint32_t ld_vol(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline void st_vol(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline void st_vol(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ inline void rel_wg() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ inline void acq_wg() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }

}  // namespace

size_t estep_df_lds_bytes(int S, int fc, int nw, int na, bool pair, int R, int qcap, int fcap) {
  return (size_t)df_plan(S, fc, na, nw - na, pair, R, qcap, fcap).bytes;
}
size_t estep_df_scratch_bytes(int fcap, int S, int R) { return (size_t)R * df_front_bytes(fcap, S); }

// WPE: resident waves per SIMD of the register allocation (4 or 5).  PAIR:
// segments of S lanes with two links per lane (S <= 16), else 2S lanes (S <= 32).
template <int WPE, bool PAIR>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE))) void estep_values_df(ValueArgs a,
                                                                                                DfPlan plan) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int S = a.S, L = a.L, hl = a.head_len;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid / WAVE;
  const int NW = blockDim.x / WAVE, NA = plan.na, NB = NW - NA;
  const int R = plan.R, qcap = plan.qcap;
  DfShared *sh = (DfShared *)(smem + plan.o_sh);
  uint32_t *queue = (uint32_t *)(smem + plan.o_queue);
  DfChain *desc = (DfChain *)(smem + plan.o_desc);
  int *ascr = (int *)(smem + plan.o_ascr);
  const int qmask = qcap - 1, qlog = plan.qlog;
  char *sp = a.scratch + (size_t)blockIdx.x * a.scratch_stride;
  const size_t hbm_slot = df_front_bytes(a.fcap, S);
  auto front = [&](int slot) {
    return VFront{smem + plan.o_front + (size_t)slot * plan.front_stride, (unsigned char *)sp + (size_t)slot * hbm_slot,
                  a.lds_fc, a.fcap, S};
  };
  auto flags = [&](int slot) { return (uint32_t *)(smem + plan.o_flags) + (size_t)slot * plan.flag_words; };
  // B waves: the selection layout of estep_values
  const int bw = wv - NA;
  const int sws = plan.sws;
  const int sps = PAIR ? sws : WAVE;
  const int bo = bw < 0 ? 0 : bw;
  const SegScratch ss{(int *)(smem + plan.o_lpos) + bo * sps, (int *)(smem + plan.o_rpos) + bo * sps,
                      (int *)(smem + plan.o_junk) + bo * (PAIR ? 4 : 2) * WAVE, (double *)(smem + plan.o_slik) + bo * sws,
                      (uint32_t *)(smem + plan.o_smeta) + bo * sws};
  const Seg sg = make_seg(PAIR ? S : 2 * S);
  const int G = plan.G;
  const int nseg = NB * G;
  const int sb = sg.g * 2 * S;
  const LinkList W{(double *)(smem + plan.o_slik), (uint32_t *)(smem + plan.o_smeta), 1};  // final selection

  __syncthreads();
  auto next_q = [&]() -> int {
    __syncthreads();
    if (tid == 0) sh->q = atomicAdd(a.next_q, 1) + (int)gridDim.x;
    __syncthreads();
    return sh->q;
  };
  // the first watchdog to fire records where (reported through cost / total)
  auto stall_note = [&](int site, int j, int val) {
    if (atomicCAS(&sh->stall_at, 0, site << 24 | wv << 16 | (j & 0xFFFF)) == 0) sh->stall_val = val;
  };
  for (int q = blockIdx.x; q < a.n_order; q = next_q()) {
    const int bi = a.order[q];
    const unsigned long long t_indiv = __builtin_amdgcn_s_memtime();
    int status0 = a.status[bi];
    if (status0 == EST_NEEDS_ORDER) status0 = EST_OK;  // the re-run of a value-only pass
    const bool pruned = status0 == EST_OK_PRUNED;      // records built with extend()'s forward test
    if (pruned) status0 = EST_OK;
    if (status0 != EST_OK) {
      if (tid == 0) {
        a.total[bi] = 0.0;
        a.ncand[bi] = 0;
        a.cost[bi] = 0;
      }
      continue;
    }
    const unsigned long long *roff = a.rec_off + (size_t)bi * (L + 1);
    for (int i = tid; i < qcap; i += blockDim.x) queue[i] = 0u;  // every slot free for lap 0
    if (tid == 0) {
      sh->q_head = 0;
      sh->q_tail = 0;
      sh->abort = 0;
      sh->status = EST_OK;
      sh->opening = hl;
      sh->a_fin = 0;
      sh->tcur = a.trace_base[bi];
      sh->stall_at = 0;
      sh->stall_val = 0;
      for (int r = 0; r < DF_RMAX; ++r) sh->ring[r].locus = -1;
    }
    __syncthreads();

    if (wv < NA) {
      // ================================================================ A ====
      const int aw = wv;  // this A wave's chains and states: blocks of 64 aw, aw + NA, aw + 2 NA, ...
      int *myascr = ascr + aw * WAVE;
      int status = EST_OK;
      bool stop = false;  // another wave stopped the individual
      // queue the entries of the lanes where `push` holds, in lane order, on
      // consecutive tickets of the block's queue
      auto enqueue = [&](bool push, uint32_t entry, const DfChain &dc) {
        const uint64_t m = wave_ballot(push);
        if (!m) return;
        int t0 = 0;
        if (lane == 0) t0 = atomicAdd(&sh->q_tail, (int)__popcll(m));
        t0 = __shfl(t0, 0);
        if (push) {
          const uint32_t t = (uint32_t)t0 + (uint32_t)__popcll(m & lanemask_lt());
          uint32_t *slot = queue + (t & (uint32_t)qmask);
          int guard = 0;
          // the slot is free for ticket t once ticket t - qcap was taken: the
          // taker leaves the next lap's empty mark (several A waves write
          // out of ticket order, so "empty" alone would let ticket t + qcap in first)
          while (ld_vol(slot) != ((t >> qlog) & 63u) << QE_LAP) {
            if (++guard > DF_SPIN_MAX || ld_vol(&sh->abort) == DF_STALL) {
              if (guard > DF_SPIN_MAX) stall_note(3, 0, (int)t);
              atomicExch(&sh->abort, DF_STALL);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (ld_vol(&sh->abort) != DF_STALL) {
            if (!(entry & QE_END)) desc[t & (uint32_t)qmask] = dc;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            st_vol(slot, entry | QE_VALID | ((t >> qlog) & 63u) << QE_LAP);
          }
        }
      };
      // wait until cond() holds; false when the individual was stopped (by
      // another wave, or by this wave's watchdog)
      auto wait_for = [&](auto cond, int site, int j, int val) -> bool {
        int guard = 0;
        while (!cond()) {
          const int ab = ld_vol(&sh->abort);
          if (ab != 0) {
            stop = true;
            return false;
          }
          if (++guard > DF_SPIN_MAX) {
            if (lane == 0) {
              stall_note(site, j, val);
              atomicExch(&sh->abort, DF_STALL);
            }
            status = EST_DF_STALL;
            return false;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        return true;
      };
      // locus j into ring slot j % R: ring info, trace record, flags cleared,
      // then the slot published (by the A wave that claimed the opening)
      auto open_locus = [&](int j) -> bool {
        const int b = j % R;
        const uint32_t *Rj = a.rec + roff[j];
        const int F = (int)Rj[0];
        const unsigned long long words = trace_locus_words((unsigned long long)F, S);
        const unsigned long long off = sh->tcur;
        if (off + words > a.trace_cap) return false;
        uint32_t *fl = flags(b);
        for (int w = lane; w < (F + 31) / 32; w += WAVE) fl[w] = 0u;
        DfRing &g = sh->ring[b];
        if (lane == 0) {
          g.rec = roff[j];
          g.tr = off;
          g.F = F;
          g.done = 0;
          sh->tcur = off + words;
          a.trace[off] = (uint32_t)F;
          a.loc_off[(size_t)bi * (L + 1) + j] = off;
        }
        wave_lds_sync();
        rel_wg();
        if (lane == 0) st_vol(&g.locus, j);
        return true;
      };
      // ---- head list (HaploPair.cpp:14-33), by A wave 0 ---------------------
      if (aw == 0 && !open_locus(hl)) {
        status = EST_OVERFLOW_TRACE;
      } else if (aw == 0) {
        const int b = hl % R;
        const uint32_t *Rh = a.rec + roff[hl];
        const int F = (int)Rh[0];
        const double *Rtp = (const double *)(Rh + 4);
        const uint32_t *Rhd = Rh + 4 + 2 * F;
        const VFront Y = front(b);
        const unsigned long long off = sh->ring[b].tr;
        uint32_t *thd = a.trace + off + 1, *tln = a.trace + trace_links(off, (uint32_t)F);
        for (int t = lane; t < F; t += WAVE) {
          const bool homo = (Rhd[t] >> 24) & 1u;
          const double tpv = Rtp[t];
          const uint32_t mw = meta_pack(0, 0, false, homo, true);
          *Y.fwd(t) = homo ? tpv : tpv * 2.0;
          Y.lik(t)[0] = tpv;
          *Y.hm(t) = homo ? 1ull : 0ull;
          *Y.nl(t) = 1;
          thd[t] = (Rhd[t] & 0xFFFFu) | 1u << 16;
          uint32_t *tl = tln + (size_t)t * S;
          tl[0] = mw;
          for (int k = 1; k < S; ++k) tl[k] = 0u;
        }
        rel_wg();
        uint32_t *fl = flags(b);
        for (int w = lane; w < (F + 31) / 32; w += WAVE) {
          const int nb = F - 32 * w;
          st_vol(fl + w, nb >= 32 ? ~0u : ((1u << nb) - 1u));
        }
        if (lane == 0) atomicAdd(&sh->ring[b].done, F);
      }
      // ---- forward over loci ------------------------------------------------
      for (int j = hl + 1; j <= L && status == EST_OK && !stop; ++j) {
        const int b = j % R, bx = (j - 1) % R;
        // locus j-1 open (for the waves other than 0: the head); the first A
        // wave here opens locus j, once the slot's previous occupant, locus
        // j - R, is complete (its last chains write into the slot) and so are
        // its readers, locus j - R + 1; the others wait for the slot
        if (!wait_for([&] { return ld_vol(&sh->ring[bx].locus) == j - 1; }, 10, j, 0)) break;
        int won = 0;
        if (lane == 0) won = atomicCAS(&sh->opening, j - 1, j) == j - 1;
        won = __shfl(won, 0);
        if (won) {
          bool ok = true;
          for (int jg = j - R; jg <= j - R + 1 && ok; ++jg) {
            if (jg < hl) continue;
            const DfRing *g = &sh->ring[jg % R];
            ok = wait_for([&] { return ld_vol(&g->done) == ld_vol(&g->F); }, 11, j, jg);
          }
          if (!ok) break;
          if (!open_locus(j)) {
            status = EST_OVERFLOW_TRACE;
            break;
          }
        } else if (!wait_for([&] { return ld_vol(&sh->ring[b].locus) == j; }, 12, j, 0)) {
          break;
        }
        acq_wg();
        const VFront X = front(bx), Y = front(b);
        const uint32_t *xfl = flags(bx);
        uint32_t *yfl = flags(b);
        const uint32_t *Rj = a.rec + roff[j];
        const int F = (int)Rj[0], C = (int)Rj[1], NCH = (int)Rj[2];
        const double *Rtp = (const double *)(Rj + 4);
        const uint32_t *Rhd = Rj + 4 + 2 * F, *Rcb = Rhd + F, *Rct = Rcb + F + 1, *Rch = Rct + C;
        const unsigned long long toff = sh->ring[b].tr;
        uint32_t *thd = a.trace + toff + 1, *tln = a.trace + trace_links(toff, (uint32_t)F);
        int st = -1, rchk = 0;  // this lane's state, its first contribution not known to be final
        // next chain position, next candidate of the sweep over the others: in
        // this wave's blocks of 64 (block k of the locus when k % NA == aw)
        int nextc = aw * WAVE, scan = aw * WAVE;
        bool underflow = false;
        int idle = 0;  // iterations in a row without a ready state (watchdog)
        while (true) {
          // ---- free lanes take states: chains first (longest first), then the rest
          uint64_t fm = wave_ballot(st < 0);
          if (fm && nextc < NCH) {
            const int rk = __popcll(fm & lanemask_lt());
            const int be = min((nextc / WAVE + 1) * WAVE, NCH);  // this block's end
            const int nt = min(__popcll(fm), be - nextc);
            if (st < 0 && rk < nt) {
              st = (int)Rch[nextc + rk];
              rchk = (int)Rcb[st];
            }
            nextc += nt;
            if (nextc % WAVE == 0) nextc += (NA - 1) * WAVE;  // block done: this wave's next one
            fm = wave_ballot(st < 0);
          }
          if (fm && nextc >= NCH && scan < F) {
            const int bend = (scan / WAVE + 1) * WAVE;
            const int t = scan + lane;
            const bool cand = t < bend && t < F && !(Rhd[t < F ? t : 0] & HDR_CHAIN);
            const uint64_t cm = wave_ballot(cand);
            const int nc = __popcll(cm), nt = min(__popcll(fm), nc);
            if (cand) myascr[__popcll(cm & lanemask_lt())] = t;
            wave_lds_sync();
            const int rk = __popcll(fm & lanemask_lt());
            if (st < 0 && rk < nt) {
              st = myascr[rk];
              rchk = (int)Rcb[st];
            }
            scan = nt < nc ? myascr[nt] : bend + (NA - 1) * WAVE;
            wave_lds_sync();
          }
          const uint64_t held = wave_ballot(st >= 0);
          if (!held) {
            if (nextc >= NCH && scan >= F) break;
            if (++idle > DF_SPIN_MAX) {
              if (lane == 0) stall_note(1, j, scan);
              status = EST_DF_STALL;
              break;
            }
            continue;
          }
          // ---- readiness: every predecessor this state reads is final
          bool ready = false;
          if (st >= 0) {
            const int ce = (int)Rcb[st + 1];
            int r = rchk;
            bool blocked = false;
            while (r < ce && !blocked) {  // four contribution words per round of loads
              uint32_t ws[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) ws[u] = r + u < ce ? Rct[r + u] : 0u;
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                if (blocked || r >= ce) break;
                const uint32_t p = cw_state(ws[u]);
                if (!((ld_vol(xfl + (p >> 5)) >> (p & 31u)) & 1u)) blocked = true;
                else ++r;
              }
            }
            rchk = r;
            ready = r == ce;
          }
          if (!wave_ballot(ready)) {
            if (ld_vol(&sh->abort) != 0) {
              stop = true;
              break;
            }
            if (++idle > DF_SPIN_MAX) {
              if (lane == 0) stall_note(2, j, st);  // (lane 0's state)
              status = EST_DF_STALL;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
          }
          idle = 0;
          acq_wg();
          // ---- phase A of estep_values for the ready states: the extension
          // constructor (HaploPair.cpp:35-61), the appends that fit (:63-84)
          // and the ordered forward sum (:42, :66)
          bool chain = false, fin = false;
          DfChain dc;
          if (ready) {
            const int t = st;
            const double tpv = Rtp[t];
            const uint32_t hd = Rhd[t];
            const bool differ = (hd & 0xFFu) != ((hd >> 8) & 0xFFu);
            const int cb = (int)Rcb[t], ce = (int)Rcb[t + 1];
            double fwd = 0.0;
            for (int rb = cb; rb < ce; rb += 4) {
              uint32_t ws[4];
              double fs[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) ws[u] = rb + u < ce ? Rct[rb + u] : Rct[cb];
#pragma unroll
              for (int u = 0; u < 4; ++u) fs[u] = *X.fwd((int)cw_state(ws[u]));
#pragma unroll
              for (int u = 0; u < 4; ++u)
                if (rb + u < ce) {
                  const double v = fs[u] * tpv;
                  fwd = rb + u == cb ? v : fwd + v;
                }
            }
            uint32_t w = Rct[cb];
            uint32_t s = cw_state(w), ns = cw_ns(w);
            double *yl = Y.lik(t);
            unsigned long long yhm = 0ull;
            uint32_t *tl = tln + (size_t)t * S;
            copy_extended_hm<4>(X.lik((int)s), *X.hm((int)s), yl, yhm, 0, (int)ns, s, tpv, cw_rev(w), differ, tl);
            int k = (int)ns, r0 = ce;
            for (int r = cb + 1; r < ce; ++r) {
              w = Rct[r];
              s = cw_state(w);
              ns = cw_ns(w);
              if (k + (int)ns <= S) {
                copy_extended_hm<4>(X.lik((int)s), *X.hm((int)s), yl, yhm, k, (int)ns, s, tpv, cw_rev(w), differ, tl);
                k += (int)ns;
              } else {
                r0 = r;
                break;
              }
            }
            if (r0 == ce)
              for (int qq = k; qq < S; ++qq) tl[qq] = 0u;
            thd[t] = (hd & 0xFFFFu) | (uint32_t)k << 16;
            *Y.fwd(t) = fwd;
            *Y.hm(t) = yhm;
            *Y.nl(t) = (uint32_t)k;
            *Y.r0(t) = (uint32_t)r0;
            if (!(fwd > 0.0) && j < L && !pruned) underflow = true;
            chain = r0 < ce;
            fin = !chain;
            if (chain) {  // w = the contribution word of add r0
              dc.tpv = tpv;
              dc.r = (uint32_t)r0;
              dc.re = (uint32_t)ce;
              dc.k0 = (uint32_t)k | (differ ? 1u << 31 : 0u);
              dc.wc = w;
              dc.wn = r0 + 1 < ce ? Rct[r0 + 1] : 0u;
            }
          }
          rel_wg();
          if (fin) atomicOr(yfl + (st >> 5), 1u << (st & 31));
          const int nfin = __popcll(wave_ballot(fin));
          if (lane == 0 && nfin) atomicAdd(&sh->ring[b].done, nfin);
          enqueue(chain, (uint32_t)b << QE_SLOT | (uint32_t)(chain ? st : 0), dc);
          if (ready) st = -1;
          if (wave_ballot(underflow)) {
            status = EST_NEEDS_EXACT;
            break;
          }
          if (ld_vol(&sh->abort) != 0) {
            stop = true;
            break;
          }
        }
      }
      if (status == EST_DF_STALL && lane == 0) atomicExch(&sh->abort, DF_STALL);
      if (status != EST_OK && lane == 0) {
        atomicCAS(&sh->status, EST_OK, status);
        atomicCAS(&sh->abort, 0, 1);
      }
      rel_wg();
      // the last A wave done queues END for every B segment (after every chain:
      // each segment has taken, or will take, one more ticket)
      int last = 0;
      if (lane == 0) last = atomicAdd(&sh->a_fin, 1) == NA - 1;
      last = __shfl(last, 0);
      if (last && ld_vol(&sh->abort) != DF_STALL)
        for (int e = 0; e < nseg; e += WAVE) enqueue(e + lane < nseg, QE_END, DfChain{});
      if (ld_vol(&sh->abort) == DF_STALL && lane == 0) sh->status = EST_DF_STALL;
    } else {
      // ================================================================ B ====
      // a segment's chain: ring slot, state, next add r of [r, re_), list
      // length k0 before the add, link words of adds r and r + 1
      int ticket = -1, cs = 0, st = 0, r = 0, re_ = 0, k0 = 0;
      bool have = false, done = sg.g >= G;
      double tpv = 0.0;
      bool differ = false;
      uint32_t wc = 0, wn = 0;
      double *slot_l = ss.slik + sb + sg.k;
      uint32_t *slot_m = ss.smeta + sb + sg.k;
      int idle = 0;  // iterations in a row with no segment at work (watchdog)
      while (true) {
        if (ld_vol(&sh->abort) == DF_STALL) break;
        const bool want = !done && !have;
        if (wave_ballot(want)) {
          int tk = ticket;
          if (want && sg.k == 0 && tk < 0) tk = atomicAdd(&sh->q_head, 1);
          tk = __shfl(tk, sg.base);
          uint32_t e = 0u;
          if (want && sg.k == 0) e = ld_vol(queue + (tk & qmask));
          e = __shfl(e, sg.base);
          ticket = want ? tk : ticket;
          const bool got = want && (e & QE_VALID) && ((e >> QE_LAP) & 63u) == (((uint32_t)tk >> qlog) & 63u);
          if (got) {
            acq_wg();
            ticket = -1;
            if (e & QE_END) {
              done = true;
            } else {
              cs = (int)((e >> QE_SLOT) & 7u);
              st = (int)(e & F_MASK);
              const DfChain dc = desc[tk & qmask];
              r = (int)dc.r;
              re_ = (int)dc.re;
              tpv = dc.tpv;
              differ = dc.k0 >> 31;
              k0 = (int)(dc.k0 & 0x7FFFFFFFu);
              wc = dc.wc;
              wn = dc.wn;
            }
          }
          wave_lds_sync();  // the descriptor is read before its slot can be reused
          if (got) {
            if (sg.k == 0)  // (only the segment's first lane read the entry) free for ticket tk + qcap
              st_vol(queue + (tk & qmask), ((((uint32_t)tk >> qlog) + 1u) & 63u) << QE_LAP);
            if (!done) {
              const DfRing &g = sh->ring[cs];
              const int F = g.F;
              const VFront Y = front(cs);
              if (sg.k < k0) {  // the partial list: likelihoods here, link words in the trace record
                *slot_l = Y.lik(st)[sg.k];
                *slot_m = a.trace[trace_links(g.tr, (uint32_t)F) + (size_t)st * S + sg.k];
              }
              have = true;
            }
          }
        }
        if (!wave_ballot(have)) {
          if (!wave_ballot(!done)) break;
          if (++idle > DF_SPIN_MAX) {
            if (lane == 0) {
              stall_note(4, 0, ld_vol(&sh->q_tail) << 16 | (ld_vol(&sh->q_head) & 0xFFFF));
              atomicExch(&sh->abort, DF_STALL);
              sh->status = EST_DF_STALL;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        idle = 0;
        int n = 0;
        if (have) {
          const VFront X = front((cs + R - 1) % R);
          const unsigned long long xhm = *X.hm((int)cw_state(wc));
          const uint32_t s = cw_state(wc), ns = cw_ns(wc);
          const bool rev = cw_rev(wc);
          n = k0 + (int)ns;
          // HaploPair::add transformation (HaploPair.cpp:63-80)
          auto extend = [&](int kk) {
            const int qk = kk - k0;
            double lk = X.lik((int)s)[qk] * tpv;
            bool homo = (xhm >> qk) & 1ull;
            if (differ && homo) {
              if (rev) lk = 0.0;
              homo = false;
            }
            slot_l[kk - sg.k] = lk;
            slot_m[kk - sg.k] = meta_pack(s, (uint32_t)qk, rev, homo, false);
          };
          if (sg.k >= k0 && sg.k < n) extend(sg.k);
          if (PAIR && sg.k + S >= k0 && sg.k + S < n) extend(sg.k + S);
          wc = wn;
          if (r + 2 < re_) {
            const DfRing &g = sh->ring[cs];
            const uint32_t *Rj = a.rec + g.rec;
            const int F = g.F;
            wn = (Rj + 4 + 2 * F + F + F + 1)[r + 2];
          } else {
            wn = 0u;
          }
        }
        wave_lds_sync();
        if (PAIR) seg2_nth_slots(n, S - 1, sg, ss);
        else seg_nth_slots(n, S - 1, sg, ss);
        if (have) {
          k0 = S;
          if (++r == re_) {  // the chain's list is final
            const DfRing &g = sh->ring[cs];
            const VFront Y = front(cs);
            const uint32_t *Rj = a.rec + g.rec;
            const int F = g.F;
            const uint32_t *Rhd = Rj + 4 + 2 * F;
            uint32_t *tl = a.trace + trace_links(g.tr, (uint32_t)F) + (size_t)st * S;
            const uint32_t fm = sg.k < S ? *slot_m : 0u;
            if (sg.k < S) {
              Y.lik(st)[sg.k] = *slot_l;
              tl[sg.k] = fm;
            }
            // the final list's homozygous flags, bit k = position k (lanes k < S of the segment)
            const unsigned long long hb = (wave_ballot(have && sg.k < S && meta_homo(fm)) >> sg.base) &
                                          (S >= 64 ? ~0ull : ((1ull << S) - 1ull));
            if (sg.k == 0) {
              *Y.hm(st) = hb;
              *Y.nl(st) = (uint32_t)S;
              a.trace[g.tr + 1 + st] = (Rhd[st] & 0xFFFFu) | (uint32_t)S << 16;
            }
            rel_wg();
            wave_lds_sync();  // the segment's stores are all issued before its flag
            if (sg.k == 0) {
              atomicOr(flags(cs) + (st >> 5), 1u << (st & 31));
              atomicAdd(&sh->ring[cs].done, 1);
            }
            have = false;
          }
        }
      }
    }
    __syncthreads();

    // ---- final selection (HaploBuilder.cpp:87-116) ------------------------
    if (tid == 0) {
      a.cost[bi] = (int32_t)((__builtin_amdgcn_s_memtime() - t_indiv) >> 10);
      int status = sh->status;
      int cnt = 0;
      double total = 0.0;
      const VFront X = front(L % R);
      const int Fp = sh->ring[L % R].F;
      if (status == EST_OK) {
        for (int t = 0; t < Fp; ++t) {
          total += *X.fwd(t);
          const uint32_t n = *X.nl(t);
          for (uint32_t k = 0; k < n; ++k) {
            double lk = X.lik(t)[k];
            const bool homo = (*X.hm(t) >> k) & 1ull;
            if (!homo) lk *= 2.0;
            W.set(cnt++, lk, meta_pack((uint32_t)t, k, false, homo, false));
          }
          if (cnt > S) {
            if (cnt <= 32) nth_element_greater_masks(W, cnt, S - 1, cnt);
            else nth_element_greater(W, cnt, S - 1);
            cnt = S;
          }
        }
        sort_greater(W, cnt, (int *)(smem + plan.o_lpos));
      }
      a.status[bi] = status;
      if (status == EST_OK) {
        double coverage = 0.0;
        for (int c = 0; c < cnt; ++c) {
          const uint32_t mm = W.m(c);
          const uint32_t t = meta_pred(mm), k = meta_idx(mm);
          const double own = X.lik((int)t)[k];
          const double prior = meta_homo(mm) ? own : own * 2.0;  // HaploPair.cpp:97-102
          const double post = prior / total;
          coverage += post;
          a.cand_state[(size_t)bi * S_MAX + c] = t;
          a.cand_idx[(size_t)bi * S_MAX + c] = k;
          a.prior[(size_t)bi * S_MAX + c] = prior;
          a.posterior[(size_t)bi * S_MAX + c] = post;
        }
        for (int c = 0; c < cnt; ++c)  // HaploModel.cpp:97-98
          a.weight[(size_t)bi * S_MAX + c] = a.posterior[(size_t)bi * S_MAX + c] / coverage;
      } else {
        cnt = 0;
      }
      a.total[bi] = total;
      a.ncand[bi] = cnt;
      if (status == EST_DF_STALL) {  // where the watchdog fired (host message)
        a.cost[bi] = sh->stall_at;
        a.total[bi] = (double)sh->stall_val;
      }
    }
    __syncthreads();
  }
}

hipError_t launch_estep_values_df(const ValueArgs &a, int grid, int nw, int na, int wpe, bool pair, int R, int qcap,
                                  hipStream_t st) {
  const int G = pair ? WAVE / a.S : WAVE / (2 * a.S);
  if (a.S < 1 || a.S > 32 || (pair && a.S > 16) || nw < 2 || nw > 16 || na < 1 || na >= nw || (wpe != 4 && wpe != 5) ||
      R < 3 || R > DF_RMAX || qcap < 64 || (qcap & (qcap - 1)) || qcap > 4096 || qcap < (nw - na) * G ||
      !a.trace_base || a.fcap > F_MAX || a.lds_fc < 0 || a.lds_fc > a.fcap)
    return hipErrorInvalidValue;
  const DfPlan plan = df_plan(a.S, a.lds_fc, na, nw - na, pair, R, qcap, a.fcap);
  const size_t lds = (size_t)plan.bytes;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    for (const void *f : {(const void *)estep_values_df<4, true>, (const void *)estep_values_df<4, false>,
                          (const void *)estep_values_df<5, true>, (const void *)estep_values_df<5, false>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
  }
  const dim3 g(grid), b(WAVE * nw);
  if (pair) {
    if (wpe == 5) hipLaunchKernelGGL((estep_values_df<5, true>), g, b, lds, st, a, plan);
    else hipLaunchKernelGGL((estep_values_df<4, true>), g, b, lds, st, a, plan);
  } else {
    if (wpe == 5) hipLaunchKernelGGL((estep_values_df<5, false>), g, b, lds, st, a, plan);
    else hipLaunchKernelGGL((estep_values_df<4, false>), g, b, lds, st, a, plan);
  }
  return hipGetLastError();
}

}  // namespace hmc
#else
namespace hmc {
size_t estep_df_lds_bytes(int, int, int, int, bool, int, int, int) { return 0; }
size_t estep_df_scratch_bytes(int, int, int) { return 0; }
hipError_t launch_estep_values_df(const ValueArgs &, int, int, int, int, bool, int, int, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace hmc
#endif  // HMC_VARIANTS
