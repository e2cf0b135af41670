// ctx.hpp — the host runtime's context (Ctx): device buffers, the panel,
// the pattern table, the E-step stores and the EM state of one rank.  The
// member functions live in ctx_panel.cpp (collectives, panel upload),
// ctx_mine.cpp (pattern search), ctx_exact.cpp (exact M-step), ctx_estep.cpp
// (E-step store planning and passes) and ctx_run.cpp (HaploComp, EM driver,
// model snapshot); api.cpp holds the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <functional>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hmc_amd.h"
#include "haplofile.hpp"
#include "hmc_internal.hpp"
#include "mstep.hpp"
#include "exact.hpp"
#include "select.hpp"

namespace hmc {

// ------------------------------------------------------------- utilities --
template <class T>
struct DevBuf {
  T *p = nullptr;
  size_t n = 0;
  bool host = false;  // pinned host memory instead (model snapshots of very large tables)
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)(host ? hipHostFree(p) : hipFree(p));
    p = nullptr;
    n = 0;
  }
  void set_host(bool h) {
    if (h != host) release();
    host = h;
  }
  hipError_t alloc(T **q, size_t bytes) {
    return host ? hipHostMalloc((void **)q, bytes, hipHostMallocDefault) : hipMalloc((void **)q, bytes);
  }
  // Contents not preserved.  A buffer that has to grow takes 1.5x headroom:
  // large allocations are mapped eagerly by the HIP runtime (~1 s per 10-20 GB),
  // so slowly growing per-level buffers must not be re-allocated every level.
  hipError_t ensure(size_t m) {
    if (m <= n && p) return hipSuccess;
    const size_t want = std::max<size_t>(m, 1), grown = n ? std::max(want, n + n / 2) : want;
    release();
    size_t got = grown;
    hipError_t e = alloc(&p, got * sizeof(T));
    if (e != hipSuccess && grown > want) {
      (void)hipGetLastError();
      got = want;
      e = alloc(&p, got * sizeof(T));
    }
    if (e != hipSuccess) { p = nullptr; return e; }
    n = got;
    return hipSuccess;
  }
  hipError_t grow_keep(size_t m, size_t used, hipStream_t st) {  // preserve the first `used` elements
    if (m <= n && p) return hipSuccess;
    size_t cap = std::max<size_t>(m, n + n / 2);
    T *q = nullptr;
    hipError_t e = hipMalloc((void **)&q, cap * sizeof(T));
    if (e != hipSuccess) return e;
    if (p && used) {
      e = hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e != hipSuccess) { (void)hipFree(q); return e; }
    }
    release();
    p = q;
    n = cap;
    return hipSuccess;
  }
};

// Page-locked host buffer for small per-level readbacks: a DtoH copy into pageable
// memory goes through a staging buffer and a second copy on every mining level.
template <class T>
struct PinnedBuf {
  T *p = nullptr;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf &) = delete;
  PinnedBuf &operator=(const PinnedBuf &) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t m) {
    if (p) return hipSuccess;
    hipError_t e = hipHostMalloc((void **)&p, std::max<size_t>(m, 1) * sizeof(T), hipHostMallocDefault);
    if (e != hipSuccess) p = nullptr;
    return e;
  }
};

struct Err {
  int code;
};

// ----------------------------------------------------------------- panel --
struct Panel {
  int N = 0, L = 0, amax = 0;
  int unphased = 0;  // GenoData::unphased_num (GenoData.h:37): HaploComp covers individuals [0, unphased)
  std::vector<int32_t> al;  // [N][2][L] symbols, -1 missing
  std::string types;
  std::vector<std::vector<std::pair<int32_t, double>>> sym;  // per locus (symbol, frequency), ascending
  std::vector<uint8_t> idx;                                  // [N][2][L] allele index, 0xFF missing

  // GenoData::checkAlleleSymbol (GenoData.cpp:78-118): distinct non-missing
  // symbols sorted by value; frequency = count / non-missing count.
  bool build_tables(std::string &err) {
    unphased = N;  // GenoData::setGenotypeNum (GenoData.cpp:46-57)
    sym.assign(L, {});
    idx.assign((size_t)N * 2 * L, MISSING);
    amax = 0;
    for (int k = 0; k < L; ++k) {
      std::map<int32_t, double> cnt;
      double tot = 0.0;
      for (int i = 0; i < N; ++i)
        for (int h = 0; h < 2; ++h) {
          const int32_t a = al[((size_t)i * 2 + h) * L + k];
          if (a >= 0) {
            cnt[a] += 1.0;
            tot += 1.0;
          }
        }
      for (auto &kv : cnt) sym[k].push_back({kv.first, kv.second / tot});
      if ((int)sym[k].size() > A_MAX) {
        err = "locus " + std::to_string(k) + " has more than " + std::to_string(A_MAX) + " alleles";
        return false;
      }
      amax = std::max(amax, (int)sym[k].size());
      for (int i = 0; i < N; ++i)
        for (int h = 0; h < 2; ++h) {
          const int32_t a = al[((size_t)i * 2 + h) * L + k];
          if (a < 0) continue;
          int j = 0;
          while (sym[k][j].first != a) ++j;
          idx[((size_t)i * 2 + h) * L + k] = (uint8_t)j;
        }
    }
    amax = std::max(amax, 1);
    return true;
  }
  int32_t symbol(int k, uint8_t j) const { return j == MISSING ? -1 : sym[k][j].first; }
  int index_of(int k, int32_t a) const {
    for (size_t j = 0; j < sym[k].size(); ++j)
      if (sym[k][j].first == a) return (int)j;
    return -1;
  }
};

// HaploFile::readGenoData (HaploFile.cpp:54-118) with AlleleSequence::read
// (Allele.cpp:55-153): ids on (the first token of the id line, :96-100),
// `P` positions line optional (default k * 1000, GenoData.cpp:59-76), marker
// names "M<k+1>", per-locus type.  ids / positions / names go to `meta` for
// writeGenoData.
inline bool read_phase(const char *path, Panel &pn, FileData &meta, std::string &err) {
  FILE *fp = fopen(path, "r");
  if (!fp) { err = std::string("Can not open file ") + path + "!"; return false; }
  auto fail = [&](const char *m) { fclose(fp); err = m; return false; };
  int n = 0, l = 0;
  if (fscanf(fp, "%d\n", &n) != 1 || fscanf(fp, "%d\n", &l) != 1 || n <= 0 || l <= 0) return fail("Invalid file type!");
  pn.N = n;
  pn.L = l;
  pn.al.assign((size_t)n * 2 * l, -1);
  std::vector<char> line((size_t)l * 32 + 4096);
  const char *D = " \t\r\n";
  if (!fgets(line.data(), (int)line.size(), fp)) return fail("Truncated file!");
  char *s = line.data() + strspn(line.data(), D);
  meta = FileData();
  meta.N = n;
  meta.L = l;
  meta.pos.resize(l);
  meta.names.resize(l);
  for (int k = 0; k < l; ++k) {
    meta.pos[k] = k * 1000;  // Constant::average_marker_distance (Constant.cpp:5)
    meta.names[k] = "M" + std::to_string(k + 1);
  }
  meta.ids.assign(n, "");
  if (s[0] == 'P') {
    s += strcspn(s, D);
    s += strspn(s, D);
    for (int k = 0; k < l; ++k) {  // setAllelePosition(i, atoi(s)) (HaploFile.cpp:80-84)
      meta.pos[k] = atoi(s);
      s += strcspn(s, D);
      s += strspn(s, D);
    }
    if (!fgets(line.data(), (int)line.size(), fp)) return fail("Truncated file!");
    s = line.data() + strspn(line.data(), D);
  }
  pn.types.assign(l, 'M');
  for (int k = 0; k < l; ++k) {
    pn.types[k] = s[0];
    if (*s) ++s;
    s += strspn(s, D);
  }
  for (int i = 0; i < n; ++i) {
    if (!fgets(line.data(), (int)line.size(), fp)) return fail("Truncated file!");  // id line
    {
      const char *t = line.data() + strspn(line.data(), D);
      meta.ids[i] = std::string(t, strcspn(t, D));  // sscanf(line, "%s", buf)
    }
    for (int h = 0; h < 2; ++h) {
      if (!fgets(line.data(), (int)line.size(), fp)) return fail("Truncated file!");
      char *b = line.data();
      for (int k = 0; k < l; ++k) {
        b += strspn(b, D);
        int32_t a;
        if (pn.types[k] == 'S') {
          a = (b[0] == '-' || b[0] == '?' || b[0] == 0) ? -1 : (int32_t)(unsigned char)b[0];
          if (*b) ++b;
        } else {
          if (b[0] == '-' || b[0] == '?') a = -1;
          else {
            int v = atoi(b);
            a = v > 0 ? v : -1;
          }
          b += strcspn(b, D);
        }
        pn.al[((size_t)i * 2 + h) * l + k] = a;
      }
    }
  }
  fclose(fp);
  return pn.build_tables(err);
}

// ---------------------------------------------------------------- context --
struct Ctx {
  int device = 0, rank = 0, world = 1;
  hipStream_t st = nullptr;
  ncclComm_t comm = nullptr;
  hmc_allreduce_fn host_fn = nullptr;  // host-callback collective (tests, gloo)
  void *host_user = nullptr;
  bool own_comm = true;  // false: the caller's RCCL communicator (hmc_ctx_create_comm)
  // Cross-rank sums (M-step candidate sums, LL, total weight): ORDERED passes
  // each running sum from rank r-1 to rank r, which continues the chain over
  // its contiguous block of items — the reference's sequential sums
  // (PatternManager.cpp:254-262, HaploModel.cpp:110, HaploData.cpp:120-126),
  // bit for bit; ALLREDUCE sums the ranks' partial sums (fewer steps, last-bit
  // drift).
  enum { RED_ORDERED = 0, RED_ALLREDUCE = 1 };
  int reduction = RED_ORDERED;
  // A one-rank context on a one-rank RCCL communicator runs every collective
  // anyway (test hook, hmc_set_force_collectives): results are
  // unchanged, so the RCCL calls can be exercised on a one-GPU machine.
  bool force_coll = false;
  bool multi() const { return world > 1 || force_coll; }
  // Point-to-point hops of the ordered chain issued by this context (sends,
  // receives, bytes received) — hmc_comm_stats.
  int64_t p2p_sends = 0, p2p_recvs = 0;
  uint64_t p2p_bytes = 0;
  DevBuf<double> d_chain_rx, d_chain_host;  // self-hop receive buffer; small host-vector collectives
  // Bounded waits on an RCCL context (hmc_set_comm_timeout): a stream sync
  // polls the communicator's asynchronous error and gives up after
  // comm_timeout_s, aborting the communicator — a dead or stalled neighbour
  // ends the run with HMC_ERCCL instead of a hang in ncclRecv.
  double comm_timeout_s = 1800.0;
  bool comm_dead = false;
  std::string comm_msg;
  std::string err;
  // parameters (HaploModel.h:15-26 with the CLI defaults of HMC.cpp:35-47)
  double min_freq_abs = 1.5, min_freq = -1.0;
  int num_patterns = -1;  // HaploModel::num_patterns (HMC.cpp:38): > 0 selects findPatternByNum
  FileData file_meta;     // ids / marker names / positions of the last hmc_load_file
  int min_len = 1, max_len = 30, sample_size = 10;
  // tuning
  static constexpr int FCAP_INIT = 2048, FCAP_BIG = 16384;
  int fcap = FCAP_INIT, fcap_user = FCAP_INIT, waves = 0;
  int ccap_mult = 8;  // structure-pass contributions per locus = ccap_mult * fcap (grows on overflow)
  bool fcap_user_set = false;  // hmc_set_tuning gave a frontier capacity: no automatic start capacity
  int lds_waves_per_cu = 8;  // E-step individuals (blocks) sharing one CU's 160 KiB LDS
  int estep_nw = 2;          // E-step waves per individual (shape sweep at cfg 3: 2:8 beats 3:4 by 25%)
  // value-pass shape (waves per individual : individuals per CU), 0 = by group
  // size (estep_split: 1:20 from 32 individuals per CU, 2:8 from 8, else 3:8);
  // structure-pass individuals per CU, 0 = by group size (12 / 8 / 4)
  int vp_nw = 0, vp_ipc = 0, s1_ipc = 0, s1_nw = 0;
  int key_probes = 16;  // structure pass: LDS probes of the key table before its HBM tier (hmc_set_key_probes)
  // diagnostics only (stderr logging, never a change of what runs): read once
  // at context creation from HMC_DEBUG_MEM / HMC_DIAG_MINE
  bool debug_mem = false, diag_mine = false;
  bool check_records = false;  // HMC_CHECK_RECORDS: validate each structure pass's records on the host
  int validate_records(const int32_t *ids, int np_, int i0);
  // Value-pass mode (hmc_set_value_mode): value-only k-best lists first and
  // the exact pass for the individuals with ties (fast), the exact pass for
  // everyone, or automatic — fast on multi-allelic panels once the model is
  // smaller than the panel (cfg 5's E2 / E3: values 792 -> 616 ms and 734 ->
  // 594 ms with 25 % of the individuals re-run; cfg 3's biallelic E2: 452 ->
  // 683 ms with 52 % re-run, profiles/r05/value_mode/), until an E-step re-runs
  // more than 35 % of its individuals.
  enum { VM_FAST = 0, VM_EXACT = 1, VM_AUTO = 2 };
  int value_mode = VM_AUTO;
  bool fast_off = false;     // auto: a value-only E-step re-ran too many individuals (reset by a panel load)
  bool last_fast = false;    // the last E-step ran the value-only pass
  int value_pair = 2;        // two links per lane in phase B: 0 never, 1 heavy groups, 2 every group (hmc_set_value_layout)
  uint64_t trace_bytes = 0, rec_bytes = 0;  // E-step store budgets (0 = automatic)

  Panel pan;
  bool have_panel = false;
  int i0 = 0, i1 = 0;  // this rank's individuals

  // device panel
  DevBuf<uchar2> d_geno_im, d_geno_lm;
  DevBuf<uint8_t> d_anum, d_npos, d_pos_allele, d_rank_of;
  DevBuf<double> d_afreq;
  DevBuf<int32_t> d_r_child_base;
  std::vector<uint8_t> h_npos, h_anum;

  // model
  int P = 0, head_len = 1;
  // HaploModel::setModel (HaploModel.cpp:26-36): 0 MV, 1 MC, 2 MA
  int model = 0, mc_order = 1;
  // head_len > 1: alleles of the head patterns and initHeadList's pairs per
  // individual of the shard (host restatement, uploaded for the E-step)
  std::vector<uint32_t> h_head_ids;
  std::vector<uint8_t> h_head_al;  // [n_head][head_len]
  DevBuf<uint8_t> d_head_al;       // [P][head_len]
  DevBuf<uint32_t> d_hf_off, d_hf_pairs;
  DevBuf<int32_t> d_hf_status;
  bool hf_valid = false;
  bool have_model = false;
  DevBuf<int32_t> t_start, t_len, t_node, t_ppat;
  DevBuf<double> t_freq, t_prefix, t_tp;
  DevBuf<uint8_t> t_last;
  DevBuf<uint32_t> t_succ, d_head_ids, d_head_pat0;
  // The table in end-locus order for the structure pass (gmodel.hip), rebuilt
  // on the first E-step after every change of the model (model_gen, below).
  DevBuf<uint32_t> g_gid, g_inv, g_succ, g_keys;
  DevBuf<double> g_tp;
  DevBuf<uint8_t> g_last;
  DevBuf<char> g_temp;
  uint64_t gmodel_gen = ~0ull;  // the model_gen the end-order table was built for
  bool end_order = true;        // hmc_set_end_order
  int ensure_gmodel();
  int n_head = 0;
  // Table generations: every new table gets a new number; the candidate tree
  // (n_* arrays: the allele strings of a mined table) belongs to tree_gen.
  uint64_t model_gen = 0, tree_gen = ~0ull, next_gen = 0;
  bool tree_ok() const { return node_cap > 0 && tree_gen == model_gen && tree_complete; }
  void new_table(bool with_tree) {
    model_gen = ++next_gen;
    if (with_tree) tree_gen = model_gen;
  }

  // mining state
  DevBuf<int32_t> n_parent, n_start, n_child_base, n_link;
  DevBuf<uint8_t> n_allele, n_flags;
  DevBuf<double> n_freq, n_prefix, n_tp, n_sum;
  DevBuf<uint32_t> n_cnt, n_size, n_pos;
  DevBuf<unsigned long long> d_mstamps;  // diagnostic build: mine_count phase cycles
  DevBuf<unsigned long long> n_list_off, n_region, d_r_region;
  size_t node_cap = 0;
  DevBuf<uint32_t> l_idx[2];
  DevBuf<double> l_val[2];
  DevBuf<unsigned long long> s_ext, d_totals, d_rm, d_rm_save;
  PinnedBuf<unsigned long long> h_totals;  // fixed 2 slots (next list slots, next nodes)
  DevBuf<int32_t> s_child;
  DevBuf<int> d_lev_begin;  // node offset of each mining level (1..maxlev) + end
  std::vector<int> h_lev_begin;
  DevBuf<char> s_tmp;
  DevBuf<uint32_t> d_rsize, d_rpos;
  DevBuf<int> d_mine_err;
  DevBuf<double> d_flag;
  unsigned long long mine_list_cap = 0;  // bytes of one level's matching lists (0 = device memory)  // set when a successor walk needed a node outside the window

  // samples (HaploData) and E-step buffers
  int H = 0;
  double total_weight = 0.0;
  bool have_samples = false;
  DevBuf<uint8_t> d_rows, d_samp_lm, d_res;
  DevBuf<double> d_w;
  DevBuf<char> d_scratch;
  DevBuf<uint32_t> d_trace;
  DevBuf<unsigned long long> d_trace_cursor, d_loc_off, d_re;
  DevBuf<double> d_total, d_prior, d_post, d_weight;
  DevBuf<int32_t> d_ncand, d_status, d_sbase, d_fmax;
  DevBuf<uint32_t> d_cstate, d_cidx, d_maxst;
  DevBuf<unsigned long long> d_stamps;
  std::vector<double> h_total;
  std::vector<int32_t> h_ncand, h_status, h_sbase;
  std::vector<int32_t> h_cost;  // E-step scheduling: per-individual cost (heaviest first)
  DevBuf<int32_t> d_cost, d_order, d_order2, d_rowmap;
  DevBuf<double> d_wslot;                               // sample weights in slot layout
  DevBuf<unsigned long long> d_tbase, d_rbase, d_rneed, d_tneed;  // per-individual store regions / needs
  std::vector<int32_t> h_rowmap;                        // dense sample h -> slot row
  std::vector<unsigned long long> h_re;
  bool have_estep = false;
  std::vector<uint8_t> best_res;  // [n][2][L] accepted resolutions (allele index), host copy
  bool have_best = false;
  bool best_on_host = false;      // best_res matches d_best
  DevBuf<uint8_t> d_best;         // the accepted resolutions on the device
  DevBuf<int32_t> d_hc_cnt, d_hc_bad;

  // split E-step (estep_split.hip): structure pass + value pass, fused
  // kernel as the exact fallback for underflowing individuals
  enum { ESTEP_SPLIT = 0, ESTEP_FUSED = 1 };
  int estep_mode = ESTEP_SPLIT;
  DevBuf<char> d_scr1, d_scr2;
  DevBuf<int32_t> d_nextq;  // dynamic-schedule counters of the structure and value passes
  DevBuf<uint32_t> d_rec;
  DevBuf<unsigned long long> d_rec_off, d_rec_cursor;
  std::vector<int32_t> h_status1, h_redo;
  DevBuf<int32_t> d_redo;
  int n_fallback = 0;  // individuals re-run on the fused kernel by the last E-step
  int n_order_redo = 0;  // individuals re-run on the exact value pass (ties) by the last E-step

  // timings
  hipEvent_t ev[8] = {};
  // cross-rank reduction of the last pattern search: device ms between the
  // first and the last collective of each mining level (the ordered chain's
  // mine_sum launches included), and the levels reduced
  double ms_red = 0;
  int n_red_levels = 0;
  bool red_timed = false;
  double ms_fwd = 0, ms_tb = 0, ms_m = 0;
  double ms_s1 = 0, ms_s2 = 0, ms_fb = 0;  // split E-step: structure, values, fused fallback
  double ms_order = 0;                     // part of ms_s2: exact value pass re-runs

  int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  int hipfail(hipError_t e, const char *where) {
    if (comm_dead) return fail(HMC_ERCCL, "%s: %s", where, comm_msg.c_str());
    if (e == hipErrorOutOfMemory) return fail(HMC_ENOMEM, "%s: %s", where, hipGetErrorString(e));
    return fail(HMC_EHIP, "%s: %s", where, hipGetErrorString(e));
  }

  int nloc() const { return i1 - i0; }
  int S() const { return sample_size > 1 ? sample_size : 1; }  // HaploBuilder.cpp:44

  // ---------------------------------------------------------- collectives --
  // Stream sync with a bounded wait.  Without an RCCL communicator (or on one
  // rank without forced collectives) this is hipStreamSynchronize.  Otherwise
  // the host polls the stream, checks ncclCommGetAsyncError between polls, and
  // after comm_timeout_s (or on an asynchronous error) aborts the communicator
  // — RCCL's kernels waiting in a receive see the abort flag and exit — and
  // returns an error that hipfail() reports as HMC_ERCCL.
  hipError_t sync_st() {
    if (comm_dead) return hipErrorUnknown;
    if (!comm || !multi()) return hipStreamSynchronize(st);
    const auto t0 = std::chrono::steady_clock::now();
    for (long spin = 0;; ++spin) {
      hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) return hipSuccess;
      if (q != hipErrorNotReady) return q;
      ncclResult_t ar = ncclSuccess;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      bool bad = ncclCommGetAsyncError(comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress;
      if (bad || el > comm_timeout_s) {
        char m[256];
        if (bad)
          snprintf(m, sizeof m, "RCCL asynchronous error: %s (communicator aborted)", ncclGetErrorString(ar));
        else
          snprintf(m, sizeof m, "rank %d: stream not drained after %.3g s (comm timeout; communicator aborted)", rank,
                   comm_timeout_s);
        comm_msg = m;
        comm_dead = true;
        ncclCommAbort(comm);  // releases kernels blocked on a peer, and frees the communicator
        comm = nullptr;
        (void)hipStreamSynchronize(st);
        (void)hipGetLastError();
        return hipErrorUnknown;
      }
      if (spin < 2000) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(spin < 20000 ? 20 : 200));
    }
  }
  int comm_ok() { return comm_dead ? fail(HMC_ERCCL, "communicator aborted earlier: %s", comm_msg.c_str()) : HMC_OK; }

  int allreduce_sum(double *dptr, size_t n) {
    if (!multi() || n == 0) return HMC_OK;
    if (host_fn) {
      std::vector<double> h(n);
      hipError_t e;
      if ((e = hipMemcpyAsync(h.data(), dptr, n * 8, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
        return hipfail(e, "allreduce");
      if (host_fn(h.data(), n, host_user) != 0) return fail(HMC_ERCCL, "host all-reduce callback failed");
      if ((e = hipMemcpyAsync(dptr, h.data(), n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "allreduce");
      return HMC_OK;
    }
    if (int rc = comm_ok()) return rc;
    ncclResult_t r = ncclAllReduce(dptr, dptr, n, ncclDouble, ncclSum, comm, st);
    if (r != ncclSuccess) return fail(HMC_ERCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
    return HMC_OK;
  }
  // Everyone receives rank `src`'s n doubles (device buffer).  RCCL:
  // ncclBroadcast; host callback: an all-reduce in which every other rank
  // contributes +0.0 (x + 0.0 == x exactly).
  int bcast(double *dptr, size_t n, int src) {
    if (!multi() || n == 0) return HMC_OK;
    if (host_fn) {
      std::vector<double> h(n, 0.0);
      hipError_t e;
      if (rank == src && ((e = hipMemcpyAsync(h.data(), dptr, n * 8, hipMemcpyDeviceToHost, st)) ||
                          (e = sync_st())))
        return hipfail(e, "bcast");
      if (host_fn(h.data(), n, host_user) != 0) return fail(HMC_ERCCL, "host collective callback failed");
      if ((e = hipMemcpyAsync(dptr, h.data(), n * 8, hipMemcpyHostToDevice, st)) || (e = sync_st()))
        return hipfail(e, "bcast");
      return HMC_OK;
    }
    if (int rc = comm_ok()) return rc;
    ncclResult_t r = ncclBroadcast(dptr, dptr, n, ncclDouble, src, comm, st);
    if (r != ncclSuccess) return fail(HMC_ERCCL, "ncclBroadcast: %s", ncclGetErrorString(r));
    return HMC_OK;
  }
  int bcast_host(double *h, size_t n, int src) {  // small host vectors
    if (!multi() || n == 0) return HMC_OK;
    if (host_fn) {
      std::vector<double> v(h, h + n);
      if (rank != src) std::fill(v.begin(), v.end(), 0.0);
      if (host_fn(v.data(), n, host_user) != 0) return fail(HMC_ERCCL, "host collective callback failed");
      std::copy(v.begin(), v.end(), h);
      return HMC_OK;
    }
    DevBuf<double> &tmp = d_chain_host;
    hipError_t e = tmp.ensure(n);
    if (e) return hipfail(e, "bcast_host");
    if ((e = hipMemcpyAsync(tmp.p, h, n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "bcast_host");
    int rc = bcast(tmp.p, n, src);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(h, tmp.p, n * 8, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
      return hipfail(e, "bcast_host");
    return HMC_OK;
  }

  // The ordered reduction's chain (RED_ORDERED): rank 0's `d` holds its local
  // sums (the caller computed them); rank r > 0 receives the running sums of
  // ranks 0..r-1 into `d` from rank r-1, runs `cont` (which continues them over
  // its own items in order), and passes them to rank r+1; rank W-1 broadcasts
  // the finals.  W-1 point-to-point hops plus one broadcast per call, instead
  // of one broadcast from every rank (W broadcasts of W-1 hops each).  The
  // host-callback transport has only an all-reduce: there each hop is an
  // all-reduce in which one rank contributes (the same chain, W collectives).
  int ordered_chain(double *d, size_t n, const std::function<int()> &cont) {
    if (!multi() || n == 0) return HMC_OK;
    int rc;
    if (host_fn) {
      for (int r = 0; r < world; ++r) {
        if (r == rank && r > 0 && (rc = cont())) return rc;
        if ((rc = bcast(d, n, r))) return rc;
      }
      return HMC_OK;
    }
    if ((rc = comm_ok())) return rc;
    ncclResult_t x;
    if (world == 1) {
      // One-rank test hook (force_coll): the chain's hop sent to this rank
      // itself — the same ncclSend / ncclRecv calls, count, dtype and stream
      // as a W > 1 hop, grouped (a self-send completes only with its receive
      // in the same group).  The receive lands in a scratch buffer poisoned
      // with NaN first, then replaces `d`: every running sum of the run has
      // travelled through RCCL's point-to-point path.
      hipError_t e;
      if ((e = d_chain_rx.ensure(n)) || (e = hipMemsetAsync(d_chain_rx.p, 0xFF, n * 8, st)))
        return hipfail(e, "ordered_chain self hop");
      if ((x = ncclGroupStart()) != ncclSuccess) return fail(HMC_ERCCL, "ncclGroupStart: %s", ncclGetErrorString(x));
      ncclResult_t xs = ncclSend(d, n, ncclDouble, 0, comm, st);
      ncclResult_t xr = ncclRecv(d_chain_rx.p, n, ncclDouble, 0, comm, st);
      x = ncclGroupEnd();
      if (xs != ncclSuccess || xr != ncclSuccess || x != ncclSuccess)
        return fail(HMC_ERCCL, "self send/recv: %s / %s / %s", ncclGetErrorString(xs), ncclGetErrorString(xr),
                    ncclGetErrorString(x));
      p2p_sends += 1;
      p2p_recvs += 1;
      p2p_bytes += n * 8;
      if ((e = hipMemcpyAsync(d, d_chain_rx.p, n * 8, hipMemcpyDeviceToDevice, st)))
        return hipfail(e, "ordered_chain self hop");
      return bcast(d, n, 0);
    }
    if (rank > 0) {
      if ((x = ncclRecv(d, n, ncclDouble, rank - 1, comm, st)) != ncclSuccess)
        return fail(HMC_ERCCL, "ncclRecv: %s", ncclGetErrorString(x));
      p2p_recvs += 1;
      p2p_bytes += n * 8;
      if ((rc = cont())) return rc;
    }
    if (rank < world - 1) {
      if ((x = ncclSend(d, n, ncclDouble, rank + 1, comm, st)) != ncclSuccess)
        return fail(HMC_ERCCL, "ncclSend: %s", ncclGetErrorString(x));
      p2p_sends += 1;
    }
    return bcast(d, n, world - 1);
  }
  // The same chain over a small host vector (LL, total weight): `cont` runs on
  // the host over the running sums received.
  int ordered_chain_host(double *h, size_t n, const std::function<void(double *)> &cont) {
    if (!multi() || n == 0) {
      cont(h);
      return HMC_OK;
    }
    if (host_fn) {
      for (int r = 0; r < world; ++r) {
        if (r == rank) cont(h);
        int rc = bcast_host(h, n, r);
        if (rc) return rc;
      }
      return HMC_OK;
    }
    DevBuf<double> &tmp = d_chain_host;  // persistent: a hipFree per E-step would synchronise the device
    hipError_t e = tmp.ensure(n);
    if (e) return hipfail(e, "ordered_chain_host");
    if (rank == 0) cont(h);
    if ((e = hipMemcpyAsync(tmp.p, h, n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "ordered_chain_host");
    int rc = ordered_chain(tmp.p, n, [&]() -> int {
      hipError_t e2;
      if ((e2 = hipMemcpyAsync(h, tmp.p, n * 8, hipMemcpyDeviceToHost, st)) || (e2 = sync_st()))
        return hipfail(e2, "ordered_chain_host");
      cont(h);
      if ((e2 = hipMemcpyAsync(tmp.p, h, n * 8, hipMemcpyHostToDevice, st))) return hipfail(e2, "ordered_chain_host");
      return HMC_OK;
    });
    if (rc) return rc;
    if ((e = hipMemcpyAsync(h, tmp.p, n * 8, hipMemcpyDeviceToHost, st)) || (e = sync_st()))
      return hipfail(e, "ordered_chain_host");
    return HMC_OK;
  }

  int allreduce_host(double *h, size_t n) {  // small host vectors
    if (!multi() || n == 0) return HMC_OK;
    if (host_fn) return host_fn(h, n, host_user) == 0 ? HMC_OK : fail(HMC_ERCCL, "host all-reduce callback failed");
    DevBuf<double> &tmp = d_chain_host;
    hipError_t e = tmp.ensure(n);
    if (e) return hipfail(e, "allreduce_host");
    if ((e = hipMemcpyAsync(tmp.p, h, n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "allreduce_host");
    int rc = allreduce_sum(tmp.p, n);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(h, tmp.p, n * 8, hipMemcpyDeviceToHost, st))) return hipfail(e, "allreduce_host");
    if ((e = sync_st())) return hipfail(e, "allreduce_host");
    return HMC_OK;
  }

  // ---------------------------------------------------------------- panel --
  // Contiguous shard of individuals, balanced by E-step cost: a
  // base of L/8 plus the heterozygous-or-missing loci of each individual; the
  // boundaries split the prefix sum evenly (identical on every rank).
  void shard(int N, int L);

  int upload_panel();

  DevPanel dev_panel() const {
    DevPanel d;
    d.N = pan.N;
    d.L = pan.L;
    d.amax = pan.amax;
    d.geno_im = d_geno_im.p;
    d.geno_lm = d_geno_lm.p;
    d.anum = d_anum.p;
    d.afreq = d_afreq.p;
    return d;
  }

  // --------------------------------------------------------------- mining --
  // The E-step's record and trace stores hold most of HBM between E-steps;
  // a miner allocation that fails gives them back and tries again.
  template <class T>
  hipError_t ensure_or_release(DevBuf<T> &b, size_t n) {
    hipError_t e = b.ensure(n);
    if (e == hipErrorOutOfMemory && (d_trace.p || d_rec.p)) {
      (void)hipGetLastError();
      d_trace.release();
      d_rec.release();
      e = b.ensure(n);
    }
    return e;
  }

  // Node window (blocked mining, mine_impl): the node arrays hold the nodes
  // with global indices [wbase, wbase + node_cap); kernels see pointers offset
  // by -wbase and use global indices.
  long long wbase = 0;
  bool tree_complete = false;  // the window holds every node of the last mined table (one block)
  bool nodes_oom = false;  // the last grow_nodes failure was an out-of-memory
  int grow_nodes(size_t need_global, size_t used_global);
  // Drop the nodes below global index `keep` (the block before the one just
  // mined): the rest moves to the front of the arrays, in chunks no longer
  // than the gap so that no copy overlaps itself.
  template <class T>
  hipError_t slide(DevBuf<T> &b, size_t gap, size_t n) {
    for (size_t o = 0; o < n; o += gap) {
      const size_t m = std::min(gap, n - o);
      hipError_t e = hipMemcpyAsync(b.p + o, b.p + gap + o, m * sizeof(T), hipMemcpyDeviceToDevice, st);
      if (e) return e;
    }
    return hipSuccess;
  }
  int slide_window(long long keep, long long end) {
    const size_t gap = (size_t)(keep - wbase), n = (size_t)(end - keep);
    if (gap == 0) return HMC_OK;
    hipError_t e = hipSuccess;
#define SL(b) if (!e) e = slide(b, gap, n);
    SL(n_parent) SL(n_start) SL(n_child_base) SL(n_link) SL(n_allele) SL(n_flags) SL(n_freq) SL(n_prefix) SL(n_tp)
    SL(n_sum) SL(n_cnt) SL(n_size) SL(n_pos) SL(n_list_off) SL(n_region)
#undef SL
    if (e) return hipfail(e, "mine window");
    wbase = keep;
    return HMC_OK;
  }

  MineArgs mine_args(bool genotype) const;

  double current_min_freq() {  // HaploModel::findPatterns (HaploModel.cpp:52-56)
    if (min_freq_abs > 0) min_freq = min_freq_abs / (2.0 * pan.N);
    return min_freq;
  }

  // PatternManager::findPatternByNum (PatternManager.cpp:44-70) runs rounds of
  // searchPattern(true) at thresholds 1.0, 0.9, 0.81, ... keeping the
  // candidates that fail a round for the next one.  Every candidate it ever
  // generates is in the plain candidate tree mined at the last round's
  // threshold, so the tree is mined on the GPU at theta_k and the rounds are
  // replayed on the host over it (bynum_replay); when a round needs an
  // extension the tree does not have, the tree is mined again deeper.
  static constexpr size_t SCRATCH_MAX = 48ull << 30;  // per-block E-step scratch of one launch, all blocks
  static constexpr int MINE_RETRY = 1000;
  static constexpr int MINE_SPLIT = 1001;  // a block ran out of device memory: re-run it narrower
  int bynum_need = 0;  // round the replay needed beyond the mined tree
  double bynum_theta_last = -1.0;  // the last findPatternByNum threshold (m_min_freq)
  // ------------------------------------------------------- exact M-step --
  // PatternManager::estimatePatterns (PatternManager.cpp:364-410) and
  // extendPatterns (:412-438) on the host, HaploBuilder::estimateFrequency
  // (HaploBuilder.cpp:274-450) on the device (exact.hip) once per round.
  struct Cands {  // candidate patterns: alleles as allele indices
    std::vector<int32_t> start, len;
    std::vector<int64_t> aoff;
    std::vector<uint8_t> al;
    std::vector<double> freq, prefix, tp;
    size_t size() const { return start.size(); }
    const uint8_t *alleles(size_t i) const { return al.data() + aoff[i]; }
    void push(int32_t s, int32_t l, const uint8_t *a, uint8_t extra, bool with_extra, double f, double pre = 1.0,
              double t = 1.0) {
      start.push_back(s);
      len.push_back(l);
      aoff.push_back((int64_t)al.size());
      al.insert(al.end(), a, a + (with_extra ? l - 1 : l));
      if (with_extra) al.push_back(extra);
      freq.push_back(f);
      prefix.push_back(pre);
      tp.push_back(t);
    }
  };
  bool exact_estimate = false;
  bool table_on_host = false;  // the pattern table came from the exact M-step (alleles below)
  Cands ht;                    // that table, id order
  std::vector<int32_t> ht_succ;  // [P][amax]
  DevBuf<int32_t> d_tr_child, d_tr_data, d_tr_root, d_xstatus, d_xfmax;
  DevBuf<unsigned> d_xspan;  // exact_span: the walk's largest per-item list span
  DevBuf<unsigned long long> d_xre, d_xacc;
  DevBuf<double> d_xscr;
  int tr_maxd = 0;
  int exact_rounds = 0;
  uint64_t exact_candidates = 0;

  // Allele-index strings of the current device table, id order: pattern i's
  // alleles at al[off[i] .. off[i] + len[i]).  Spelled from the prefix ids
  // (ppat; a prefix precedes its extensions in DFS order), or from the
  // candidate tree where a prefix is no pattern (min_len > 1).  Fails with
  // HMC_EUNSUPPORTED when neither can spell the table (an injected table).
  int spell_table(const std::vector<int32_t> &ln, std::vector<int64_t> &off, std::vector<uint8_t> &al);

  // The current table with allele strings (mined: spelled from the prefix
  // ids; exact: the host copy).
  int table_to_host(Cands &c, std::vector<int32_t> &succ);

  // One round: HaploBuilder::estimateFrequency(patterns) for c[b, e) —
  // ForwardPatternTree, then every individual of the shard through the
  // structure pass (forward links), exact_fb and exact_walk; fixed-point
  // sums over ranks; freq / prefix / tp as at HaploBuilder.cpp:317-331.
  int estimate_round(Cands &c, size_t b, size_t e);
  size_t xacc_nc = 0;

  // exact_fb + exact_walk over the group d_order2[0, k) (structure records in place)
  int exact_group(const int32_t *ids, int k, const std::function<int(std::vector<int32_t> &)> &rerun = nullptr);
  // The trie walk of one group (the current round's trie).
  int exact_walk_group(ExactArgs &x, int k, int dev_cu);
  // Breadth-first (default): work units of one trie node each, lane by lane
  // (exact_walk_units), level by level over batches of items.
  int exact_walk_bfs(ExactArgs &x, int k, int dev_cu);
  DevBuf<int32_t> d_xu_q, d_xu_start, d_xu_node, d_xdef, d_xidx;
  DevBuf<double> d_xu_freq, d_xe_w, d_xlacc;
  DevBuf<unsigned long long> d_xu_e0, d_xcur;
  DevBuf<uint32_t> d_xu_ne, d_xe_t, d_xlbits;
  DevBuf<int> d_xndef;
  long long xw_units = 0, xw_launches = 0, xw_defers = 0;  // walk statistics of the last exact M-step
  int exact_pruned = 0;  // individuals the last exact M-step walked over pruned records (underflow)
  double ms_walk = 0;
  // Rounds of one exact M-step share the E-step model: when a round's
  // individuals ran as one structure pass and one group, the next rounds walk
  // their new tries over the same records and fwd/bwd sums (exact_walk only).
  bool xc_reuse = false;
  int xc_groups = 0, xc_fmax = 1, xc_k = 0;

  // Successors of a pattern set (PatternManager::initialize, :308-317):
  // successor[j] = the longest stored suffix of (pattern + allele j) with start
  // >= the pattern's start; found through a trie of the set per start locus.
  void host_successors(const Cands &c, std::vector<int32_t> &succ);

  // Install a host-built table (id order) on the device: SoA, successors,
  // heads (PatternManager.cpp:293-318).
  int install_host_table(Cands &c, std::vector<int32_t> &succ);

  // PatternManager::estimatePatterns (PatternManager.cpp:364-410).
  int estimate_patterns(int *P_out, uint64_t *rm_out);

  int mine(int *P_out, uint64_t *rm_out);
  static double bynum_theta(int r) {  // m_min_freq of round r: 1.0 then *= 0.9
    double t = 1.0;
    for (int i = 1; i < r; ++i) t *= 0.9;
    return t;
  }

  // Start loci per mining block (hmc_set_mine_block; 0 = automatic).  The
  // roots of the DFS are independent (PatternManager.cpp:90-108), so the
  // search can run over blocks of start loci from L-1 down: pattern ids stay
  // the DFS pre-order (a block's ids follow those of the blocks above it).  A
  // node's suffix link starts one locus later, so it lies in its own block or
  // the one above; successors are taken level by level from the first suffix
  // that is a pattern (mine_succ_level), so the node arrays hold two blocks
  // and the matching lists one, whatever the pattern lengths.  One block when
  // the panel is small or the rules need the whole tree (findPatternByNum,
  // heads longer than 1, whose patterns are not suffix-closed).
  int mine_block_starts = 0;
  double last_mine_window_gb = 0;  // node arrays' size at the end of the last search
  int block_width(int L, int mxl, int mnl, int bynum_rounds) const {
    if (bynum_rounds > 0 || mnl > 1) return L;
    int w = mine_block_starts;
    if (w <= 0) {  // about 2.5e7 individual-loci of panel per block (cfg 3: one block; cfg 4: 10)
      const double work = (double)pan.N * (double)L;
      const int nb = (int)std::ceil(work / 2.5e7);
      if (nb <= 1) return L;
      w = (L + nb - 1) / nb;
    }
    return w >= L ? L : std::max(w, 1);
  }

  // A search that fails after its first block has started has overwritten
  // part of the table (rows, node window): the context then holds no model
  // and no candidate tree, so no later E-step or spelling runs on a half-built
  // table.
  bool mine_touched = false;
  int mine_impl(int *P_out, uint64_t *rm_out, int bynum_rounds) {
    mine_touched = false;
    const int rc = mine_impl_body(P_out, rm_out, bynum_rounds);
    if (rc != HMC_OK && mine_touched) {
      have_model = false;
      tree_gen = ~0ull;
      model_gen = ++next_gen;
    }
    return rc;
  }
  int mine_impl_body(int *P_out, uint64_t *rm_out, int bynum_rounds);
  int last_mine_blocks = 0;
  long long last_mine_nodes = 0;

  struct MineBlock {
    long long first_node = 0, end_node = 0;  // global node range of the block
    long long patterns = 0;
  };

  // The level-synchronous search for the roots [lo, hi): nodes appended at
  // global index `node0`, pattern ids from `id_base`; then the block's table
  // rows, successors and (lo == 0) the head list.
  int mine_block(int lo, int hi, int mxl, int mnl, double mf, int bynum_rounds, long long node0, long long id_base,
                 MineBlock &mb, uint64_t &rm_bynum);

  int alloc_table(int np) {
    hipError_t e;
    const size_t n = std::max(np, 1);
    if ((e = t_start.ensure(n)) || (e = t_len.ensure(n)) || (e = t_node.ensure(n)) || (e = t_freq.ensure(n)) ||
        (e = t_prefix.ensure(n)) || (e = t_tp.ensure(n)) || (e = t_last.ensure(n)) || (e = t_ppat.ensure(n)) ||
        (e = t_succ.ensure(n * pan.amax)))
      return hipfail(e, "alloc_table");
    return HMC_OK;
  }
  // Grow the table to n rows keeping the first `used` (blocked mining appends blocks).
  int grow_table(size_t n, size_t used);
  PatternTable table() const;

  // Head list (PatternManager.cpp:304-306) and the locus-0 lookup used by
  // initHeadList's findLongestMatchPattern(head_len, ...) for head_len == 1.
  int set_heads(const std::vector<std::pair<uint32_t, uint8_t>> &heads /* (id, allele at 0) */);

  // The rounds of findPatternByNum over the candidate tree mined at
  // theta(rounds): acceptance order, the last round sorted by frequency
  // (std::sort, HaploPattern::greater_frequency) and cut; then node flags and
  // positions so that mine_emit / mine_succ build the table in that order.
  int bynum_replay(const MineArgs &, int ntot, int mnl, int mxl, int, uint64_t &rm_out);

  int build_heads_from_nodes(const MineArgs &, int hb, int he);

  // initHeadList (HaploBuilder.cpp:153-224) for head_len > 1, on the host: the
  // head pairs of every individual of the shard, in the reference's order
  // (head list in id order; allele sequences expanded locus by locus;
  // findLongestMatchPattern(head_len, as) must give a start-0 pattern).
  int build_head_frontier();

  // ---------------------------------------------------------------- E-step --
  // HaploModel::resolveAll (HaploModel.cpp:79-115) over this rank's shard.
  //
  // Store sizing.  Each individual keeps its structure records (split E-step)
  // and its k-best trace until its traceback; at the first E-step of a large
  // panel they exceed HBM (cfg 3: ~10^11 links), so individuals pass in groups.
  // The structure pass reports every individual's exact record and trace
  // words; an individual whose records do not fit the store keeps walking its
  // loci without writing (status EST_OVERFLOW_REC), so one pass learns every
  // size.  Groups are then cut from the heaviest-first order by prefix sums,
  // each individual gets its own region of both stores, and no pass is re-run.
  // Sample rows go to fixed slots (2*S per individual) and are gathered into
  // the reference's sample order (individuals in order, HaploModel.cpp:105-106)
  // by the transpose that builds the locus-major samples.
  int estep(double *ll_out, int *H_out, uint64_t *re_out);

  static constexpr int ESTEP_RESTART = 1;
  std::vector<unsigned long long> prev_rneed;  // records per individual of the last E-step (estimates)
  int prev_P = 0;
  DevBuf<unsigned long long> d_recsz;  // [n] record region size of each individual
  uint64_t trace_budget = 0, rec_budget = 0;  // words
  int n_struct_passes = 0, n_value_passes = 0;

  // Pass scratch, allocated while the stores hold most of HBM: on a failure
  // the trace store (dead before a value pass is launched) and, when
  // `rec_dead`, the record store give their memory back; the caller
  // re-ensures them afterwards.
  uint64_t rec_words = 0;
  hipError_t scratch_ensure(DevBuf<char> &b, size_t bytes, bool rec_dead, bool trace_dead) {
    hipError_t e = b.ensure(bytes);
    if (e != hipErrorOutOfMemory || !trace_dead) return e;
    (void)hipGetLastError();
    d_trace.release();
    if ((e = b.ensure(bytes)) != hipErrorOutOfMemory || !rec_dead) return e;
    (void)hipGetLastError();
    d_rec.release();
    return b.ensure(bytes);
  }

  // Grow a store (contents dropped) to hold `words`, within `budget`.
  int ensure_store(DevBuf<uint32_t> &b, uint64_t words, uint64_t budget, const char *what);

  EstepArgs estep_args(int S);

  int upload_order(DevBuf<int32_t> &d, const int32_t *v, int k) {
    hipError_t e;
    if (k > 0 && ((e = hipMemcpyAsync(d.p, v, (size_t)k * 4, hipMemcpyHostToDevice, st)) ||
                  (e = sync_st())))
      return hipfail(e, "estep order");
    return HMC_OK;
  }

  // Traceback of the individuals in d_order2[0, k) into their sample slots.
  int traceback_group(int k);

  int read_status(const std::vector<int32_t> &ids, int k, bool ncand, const int32_t *dstatus = nullptr) {
    // per-individual status (and candidate counts) of ids[0, k): whole arrays, small
    hipError_t e;
    const int n = nloc();
    if ((e = hipMemcpyAsync(h_status.data(), dstatus ? dstatus : d_status.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (ncand && (e = hipMemcpyAsync(h_ncand.data(), d_ncand.p, (size_t)n * 4, hipMemcpyDeviceToHost, st))) ||
        (e = sync_st()))
      return hipfail(e, "estep status");
    (void)ids;
    (void)k;
    return HMC_OK;
  }

  // Fused single-pass E-step (estep.hip) over `pending`: trace sizes are not
  // known in advance, so groups are tried and halved on a trace overflow.
  int estep_fused(const std::vector<int32_t> &order);

  // Split E-step (estep_split.hip): structure pass, value pass, fused fallback
  // for individuals whose forward likelihood underflows.
  // exact = true: the exact M-step's pass over the individuals (structure
  // records with forward links, then exact_fb + exact_walk per group instead
  // of the value pass and traceback; E-step outputs are left untouched).
  int estep_split(const std::vector<int32_t> &order, bool exact = false);

  // ---- windowed E-step (ctx_window.cpp) ----------------------------------
  // When an individual's records and traces for all loci are too large for
  // the stores to hold more than a few groups at once (cfg 4's per-rank E1 on
  // the genotype-mined M0: ~250 MB of records and ~390 MB of traces per
  // individual, groups of ~280 on 256 CUs; cfg 3's E1: five groups), the loci
  // are cut into windows.  Per window, the structure pass and the value pass
  // over the whole group, each starting from the frontier the window before
  // left in a checkpoint (pattern pairs and list lengths; forward likelihoods
  // and the k-best lists) and saving its own last frontier; the last window
  // makes the final selection.  Full traces are kept for two windows; after
  // each window the one before it is collected into survivor nodes
  // (estep_trace_gc), and the traceback (HaploPair::getGenotype,
  // HaploPair.cpp:91-124) walks the last two windows' traces and then the
  // nodes.  Bit-identical to the classic passes.
  enum { WIN_AUTO = 0, WIN_NEVER = 1, WIN_ALWAYS = 2 };
  int window_mode = WIN_AUTO;  // hmc_set_estep_windows
  int window_loci = 0;         // record indices per window (0 = from the budgets)
  DevBuf<uint32_t> d_ck[2];  // checkpoint slots: window w reads slot w & 1, writes slot (w + 1) & 1
  DevBuf<unsigned long long> d_ck_off, d_ck_cursor;
  DevBuf<uint32_t> d_nodes, d_bnd_n, d_gc_scr;  // trace survivors (3 words per node), boundary list lengths, collection scratch
  DevBuf<unsigned long long> d_bnd_off, d_node_cursor;
  DevBuf<int32_t> d_gc_order, d_gc_status, d_gc_nextq;  // the collection's own order, statuses and work counter
  double win_scale = 1.0;  // shrinks the windows after a trace store overflow (the E-step restarts)
  int last_windows = 0, last_window_loci = 0, last_window_groups = 0;  // hmc_last_estep_windows
  int n_restarts = 0;  // restarts of the last E-step (capacity growth, smaller windows): hmc_last_estep_restarts
  double ms_ck = 0;  // device ms of the trace collections (part of ms_s2)
  // Host wall time of the last EM iteration's phases (hmc_last_host_phases):
  // the E-step call, its store (re)allocation and end-order table build, the
  // sample gather after the passes, accept + HaploComp, the M-step call.
  enum { HP_ESTEP, HP_STORES, HP_GMODEL, HP_SAMPLES, HP_ACCEPT, HP_HAPLOCOMP, HP_MSTEP, HP_SETUP, HP_N };
  double hp_ms[HP_N] = {};
  struct HpTimer {
    double &acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit HpTimer(double &a) : acc(a) {}
    ~HpTimer() { acc += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
  };
  // A probe of the first loci of a sample decides: WIN_DECLINED when the
  // classic passes fit groups of at least two individuals per CU (or the
  // whole shard).
  static constexpr int WIN_DECLINED = 2;
  int estep_windowed(const std::vector<int32_t> &order);
  bool windows_allowed() const;

  // PatternManager::checkFrequency (PatternManager.cpp:146-193) of n given
  // candidates of one length against the current items (genotypes while no
  // samples exist, else the weighted samples): the per-level seam of the
  // reference's DFS (searchPattern, :100-144).  Sums in item order; across
  // ranks in rank order (or one all-reduce), as the mining levels.
  DevBuf<int32_t> d_lv_start;
  DevBuf<uint8_t> d_lv_al;
  DevBuf<double> d_lv_sum;
  int mine_level(int level, int n, const int32_t *start, const int32_t *alleles, double *freq, uint64_t *scanned);

  // LDS tiers of pass 1 (one wave per individual, `budget` bytes): states per
  // frontier, key slots (2x, power of two), contributions per locus (2x).
  // structure pass: 2 = estep_structure2 (fewer block hand-offs per locus), 1 = estep_structure
  int structure_pass_version = 1;  // hmc_set_structure_pass
  // exact M-step walk (hmc_set_exact_walk): 1 depth-first, one item per
  // wavefront (default); 4 four items per wavefront, 2 breadth-first lane
  // units (both variants)
  int exact_ipw = 1;
  // LDS split of a structure-pass block: states per frontier (fc), key slots
  // (hc, a power of two) and contributions (cc) per locus.  Key slots and
  // contributions as multiples of the states: s1_kmul / s1_cmul (tenths),
  // hmc_set_structure_tier; 0 = the defaults below.
  int s1_kmul = 0, s1_cmul = 0;
  void s1_tier(int budget, int amax, int nw, int &fc, int &hc, int &cc, bool v2 = false) const {
    // 4-wave blocks keep their lane masks out of the slots (estep_split.hip
    // k1_lid), so their 20-byte slots take a table of 4x the states: load <= 0.25
    const int km = s1_kmul > 0 ? s1_kmul : (!v2 && nw == 4 ? 40 : 20), cm = s1_cmul > 0 ? s1_cmul : 20;
    for (int f = 2048; f >= 16; f -= 16) {
      const int h = next_pow2(std::max(16, km * f / 10)), c = std::max(16, cm * f / 10);
      const size_t b = v2 ? estep_s1v2_lds_bytes(f, h, c, amax, nw) : estep_s1_lds_bytes(f, h, c, amax, nw);
      if ((int)b <= budget) { fc = f; hc = h; cc = c; return; }
    }
    fc = 0;
    hc = 16;
    cc = 0;
  }
  // Shape of the dataflow value pass: waves per individual (one A wave, the
  // rest B), individuals per CU, ring slots, queue slots, LDS states per slot.
  // False when it cannot run (LDS for the flags and one slot's tier).
  enum { VP_AUTO = 0, VP_CLASSIC = 1, VP_DATAFLOW = 2 };
  int value_pass = VP_AUTO;  // hmc_set_value_pass
  int df_ring = 3;
  int df_na = 0;  // A waves of the dataflow pass (hmc_set_dataflow_waves), 0 = by the shape
  bool last_value_df = false;
  struct DfShape {
    int nw = 0, na = 1, ipc = 0, R = 3, qcap = 64, fc = 0;
  };
  bool df_auto(bool heavy) const { (void)heavy; return false; }
  bool df_shape(int S, bool pair, bool heavy, bool small_heavy, int per_cu, int fgrp, DfShape &d) const;

  // LDS tier of pass 2: states per frontier for the block's LDS share.
  static int s2_tier(int S, int nw, int ipc, bool pair = false) {
    const int budget = 160 * 1024 / std::max(1, ipc) - 256;
    for (int f = 4096; f >= 4; f -= 4)
      if ((int)estep_s2_lds_bytes(S, f, nw, pair) <= budget) return f;
    return 0;
  }

  // Largest LDS frontier tier that fits lds_waves_per_cu waves per CU.
  // Largest LDS frontier tier for the block's LDS share; the LDS key table
  // gets at least `key_factor` x fc slots (a power of two).
  int lds_key_factor = 1;
  void lds_tier(int S, int &fc, int &hc) const {
    const int budget = 160 * 1024 / std::max(1, lds_waves_per_cu) - 256;
    fc = 0;
    hc = 64;
    const int kf = lds_key_factor;
    for (int f = 4096; f >= 0; f -= 4) {
      const int h = next_pow2(std::max(64, kf * f));
      if ((int)estep_lds_bytes(S, f, h, estep_nw, pan.amax) <= budget) { fc = f; hc = h; return; }
    }
  }

  static int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
  }

  DevModel dev_model() const;

  // selected pairs of the last E-step, allele indices [n][2][L]
  int resolutions_idx(std::vector<uint8_t> &out);

  void to_symbols(const std::vector<uint8_t> &idx, int32_t *out) const {
    const int n = nloc(), L = pan.L;
    for (int i = 0; i < n; ++i)
      for (int h = 0; h < 2; ++h)
        for (int k = 0; k < L; ++k) {
          const size_t o = ((size_t)i * 2 + h) * L + k;
          out[o] = pan.symbol(k, idx[o]);
        }
  }

  // ------------------------------------------------------------ HaploComp --
  // HaploComp compare(&genos, &resolutions) (HaploComp.cpp:29-76, 144-155;
  // HaploModel.cpp:134): the input panel as given (the "real" phase) against
  // res = [n][2][L] allele indices of this rank's individuals.  Integer
  // counters, summed over ranks (HaploComp::operator+=, :78-90), then
  // out = {switch error, IHP, IGP}.  m_genos_input == m_genos_real there, so
  // no missing error.
  int haplocomp(double out[3]);

  // the accepted resolutions on the host (outputs)
  int sync_best() {
    if (best_on_host) return HMC_OK;
    hipError_t e;
    best_res.resize((size_t)nloc() * 2 * pan.L);
    if ((e = hipMemcpyAsync(best_res.data(), d_best.p, best_res.size(), hipMemcpyDeviceToHost, st)) ||
        (e = sync_st()))
      return hipfail(e, "resolutions");
    best_on_host = true;
    return HMC_OK;
  }

  // ------------------------------------------------------------------ run --
  // resolutions = unphased (HaploModel.cpp:127)
  int init_best();
  // HaploModel.cpp:132-133: resolutions = this E-step's best pairs (device copy)
  int accept_resolutions() {
    HpTimer hpt(hp_ms[HP_ACCEPT]);
    if (!have_estep) return fail(HMC_EARG, "no E-step has run");
    const int n = nloc(), L = pan.L;
    hipError_t e;
    if ((e = d_best.ensure((size_t)n * 2 * L)) ||
        (e = launch_gather_resolutions(d_rows.p, L, d_sbase.p, d_ncand.p, d_geno_im.p, i0, n, d_best.p, st)))
      return hipfail(e, "resolutions");
    best_on_host = false;
    return HMC_OK;
  }

  // One iteration of HaploModel::run (HaploModel.cpp:130-144): E-step, accept
  // the resolutions if the LL did not drop, HaploComp, the continue rule, and
  // the M-step when continuing (or always, force_m: a fixed number of steps).
  int em_iteration(int it, int max_iter, bool force_m, double &old_ll, hmc_iter_log &rec, bool &go);

  // ------------------------------------------------------- model snapshot --
  // A device copy of one pattern table (hmc_model_save) and the rewind of the
  // EM to the state right after the M-step that built it (hmc_em_rewind):
  // HaploModel::run after build() (HaploModel.cpp:121-129) — no samples,
  // resolutions = the input genotypes, nothing learned from earlier E-steps
  // (scheduling costs, store-size estimates, frontier capacity).  Lets a host
  // run the reference's converged chain from M0 repeatedly without mining M0
  // again (bench.py).
  struct Snap {
    bool valid = false, table_on_host = false;
    int P = 0, head_len = 1, n_head = 0;
    int L = 0, amax = 0;  // the panel's shape when saved (successor rows are amax wide)
    uint64_t gen = 0;
    DevBuf<int32_t> start, len, node, ppat;
    DevBuf<double> freq, prefix, tp;
    DevBuf<uint8_t> last, head_al;
    DevBuf<uint32_t> succ, head_ids, head_pat0;
    std::vector<uint32_t> h_head_ids;
    std::vector<uint8_t> h_head_al;
    Cands ht;
    std::vector<int32_t> ht_succ;
  } snap;

  template <class T>
  hipError_t dcopy(DevBuf<T> &dst, const DevBuf<T> &src, size_t n) {
    if (n == 0 || !src.p) return hipSuccess;
    hipError_t e = dst.ensure(n);
    if (e) return e;
    return hipMemcpyAsync(dst.p, src.p, n * sizeof(T), hipMemcpyDefault, st);
  }
  int model_save();
  int em_rewind();

  int run(int max_iter, hmc_iter_log *log, int cap, int *iters, double *t_m0, uint64_t *rm0, int *np0);
};

}  // namespace hmc
