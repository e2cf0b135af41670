// api.cpp — host runtime of libhmc_amd.so: the C-ABI of include/hmc_amd.h,
// the HaploModel EM driver, GenoData construction and PHASE I/O.
//
// Roles kept from the reference (drop-in seams):
//   GenoData::checkAlleleSymbol   GenoData.cpp:78-118        -> Panel::build_tables
//   HaploFile::readGenoData       HaploFile.cpp:54-118       -> read_phase
//   HaploFile::writeGenoData      HaploFile.cpp:120-153      -> hmc_write_phase
//   PatternManager::findPatternByFreq + initialize            -> Ctx::mine (mstep.hip)
//   HaploModel::resolveAll        HaploModel.cpp:79-115      -> Ctx::estep (estep.hip)
//   HaploModel::run               HaploModel.cpp:117-155     -> Ctx::run
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
static bool read_phase(const char *path, Panel &pn, FileData &meta, std::string &err) {
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
  // diagnostics only (stderr logging, never a change of what runs): read once
  // at context creation from HMC_DEBUG_MEM / HMC_DIAG_MINE
  bool debug_mem = false, diag_mine = false;
  bool value_fast = false;   // value-only k-best lists first, the exact pass for ties only (hmc_set_value_mode)
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
  hipEvent_t ev[6] = {};
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
    if (e == hipErrorOutOfMemory) return fail(HMC_ENOMEM, "%s: %s", where, hipGetErrorString(e));
    return fail(HMC_EHIP, "%s: %s", where, hipGetErrorString(e));
  }

  int nloc() const { return i1 - i0; }
  int S() const { return sample_size > 1 ? sample_size : 1; }  // HaploBuilder.cpp:44

  // ---------------------------------------------------------- collectives --
  int allreduce_sum(double *dptr, size_t n) {
    if (!multi() || n == 0) return HMC_OK;
    if (host_fn) {
      std::vector<double> h(n);
      hipError_t e;
      if ((e = hipMemcpyAsync(h.data(), dptr, n * 8, hipMemcpyDeviceToHost, st)) || (e = hipStreamSynchronize(st)))
        return hipfail(e, "allreduce");
      if (host_fn(h.data(), n, host_user) != 0) return fail(HMC_ERCCL, "host all-reduce callback failed");
      if ((e = hipMemcpyAsync(dptr, h.data(), n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "allreduce");
      return HMC_OK;
    }
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
                          (e = hipStreamSynchronize(st))))
        return hipfail(e, "bcast");
      if (host_fn(h.data(), n, host_user) != 0) return fail(HMC_ERCCL, "host collective callback failed");
      if ((e = hipMemcpyAsync(dptr, h.data(), n * 8, hipMemcpyHostToDevice, st)) || (e = hipStreamSynchronize(st)))
        return hipfail(e, "bcast");
      return HMC_OK;
    }
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
    DevBuf<double> tmp;
    hipError_t e = tmp.ensure(n);
    if (e) return hipfail(e, "bcast_host");
    if ((e = hipMemcpyAsync(tmp.p, h, n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "bcast_host");
    int rc = bcast(tmp.p, n, src);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(h, tmp.p, n * 8, hipMemcpyDeviceToHost, st)) || (e = hipStreamSynchronize(st)))
      return hipfail(e, "bcast_host");
    return HMC_OK;
  }

  int allreduce_host(double *h, size_t n) {  // small host vectors
    if (!multi() || n == 0) return HMC_OK;
    if (host_fn) return host_fn(h, n, host_user) == 0 ? HMC_OK : fail(HMC_ERCCL, "host all-reduce callback failed");
    DevBuf<double> tmp;
    hipError_t e = tmp.ensure(n);
    if (e) return hipfail(e, "allreduce_host");
    if ((e = hipMemcpyAsync(tmp.p, h, n * 8, hipMemcpyHostToDevice, st))) return hipfail(e, "allreduce_host");
    int rc = allreduce_sum(tmp.p, n);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(h, tmp.p, n * 8, hipMemcpyDeviceToHost, st))) return hipfail(e, "allreduce_host");
    if ((e = hipStreamSynchronize(st))) return hipfail(e, "allreduce_host");
    return HMC_OK;
  }

  // ---------------------------------------------------------------- panel --
  // Contiguous shard of individuals, balanced by E-step cost: a
  // base of L/8 plus the heterozygous-or-missing loci of each individual; the
  // boundaries split the prefix sum evenly (identical on every rank).
  void shard(int N, int L) {
    if (world == 1) { i0 = 0; i1 = N; return; }
    std::vector<double> pre((size_t)N + 1, 0.0);
    for (int i = 0; i < N; ++i) {
      int h = 0;
      for (int k = 0; k < L; ++k) {
        const uint8_t x = pan.idx[((size_t)i * 2) * L + k], y = pan.idx[((size_t)i * 2 + 1) * L + k];
        h += (x != y || x == MISSING) ? 1 : 0;
      }
      pre[i + 1] = pre[i] + L / 8.0 + h;
    }
    auto cut = [&](int r) {
      if (r <= 0) return 0;
      if (r >= world) return N;
      const double target = pre[N] * r / world;
      return (int)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
    };
    i0 = cut(rank);
    i1 = cut(rank + 1);
  }

  int upload_panel() {
    const int N = pan.N, L = pan.L, A = pan.amax;
    shard(N, L);
    std::vector<uchar2> im((size_t)N * L), lm((size_t)L * N);
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < L; ++k) {
        uchar2 g = make_uchar2(pan.idx[((size_t)i * 2) * L + k], pan.idx[((size_t)i * 2 + 1) * L + k]);
        im[(size_t)i * L + k] = g;
        lm[(size_t)k * N + i] = g;
      }
    h_anum.assign(L + 1, 0);
    h_npos.assign(L + 1, 0);
    std::vector<double> af((size_t)L * A, 0.0);
    std::vector<uint8_t> pa((size_t)L * A, 0xFF), rk((size_t)L * A, 0xFF);
    std::vector<int32_t> rcb(L + 1, 0);
    int tot = 0;
    for (int k = 0; k < L; ++k) {
      h_anum[k] = (uint8_t)pan.sym[k].size();
      for (size_t j = 0; j < pan.sym[k].size(); ++j) {
        af[(size_t)k * A + j] = pan.sym[k][j].second;
        if (pan.sym[k][j].second > 0) {
          pa[(size_t)k * A + h_npos[k]] = (uint8_t)j;
          rk[(size_t)k * A + j] = h_npos[k];
          h_npos[k]++;
        }
      }
      rcb[k] = tot;
      tot += h_npos[k];
    }
    rcb[L] = tot;
    hipError_t e;
#define UP(buf, vec)                                                                              \
  if ((e = buf.ensure(vec.size())) ||                                                             \
      (e = hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice, st))) \
    return hipfail(e, "upload_panel");
    UP(d_geno_im, im);
    UP(d_geno_lm, lm);
    UP(d_anum, h_anum);
    UP(d_npos, h_npos);
    UP(d_afreq, af);
    UP(d_pos_allele, pa);
    UP(d_rank_of, rk);
    UP(d_r_child_base, rcb);
#undef UP
    if ((e = hipStreamSynchronize(st))) return hipfail(e, "upload_panel");
    have_panel = true;
    have_model = have_samples = have_estep = have_best = false;
    snap.valid = false;  // a saved table belongs to the panel it was built on
    P = 0;
    H = 0;
    return HMC_OK;
  }

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
  int grow_nodes(size_t need_global, size_t used_global) {
    const size_t need = need_global - (size_t)wbase, used = used_global - (size_t)wbase;
    if (need <= node_cap) return HMC_OK;
    // doubling (each growth re-maps and copies 15 arrays)
    size_t cap = std::max<size_t>(need, 2 * node_cap);
    hipError_t e;
#define G(b)                                                                 \
  if ((e = b.grow_keep(cap, used, st)) == hipErrorOutOfMemory && (d_trace.p || d_rec.p)) { \
    (void)hipGetLastError();                                                   \
    d_trace.release();                                                         \
    d_rec.release();                                                           \
    e = b.grow_keep(cap, used, st);                                            \
  }                                                                            \
  if (e) { nodes_oom = e == hipErrorOutOfMemory; return hipfail(e, "grow_nodes"); }
    G(n_parent) G(n_start) G(n_child_base) G(n_link) G(n_allele) G(n_flags) G(n_freq) G(n_prefix) G(n_tp) G(n_sum)
    G(n_cnt) G(n_size) G(n_pos) G(n_list_off) G(n_region)
#undef G
    node_cap = cap;
    return HMC_OK;
  }
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

  MineArgs mine_args(bool genotype) const {
    MineArgs a;
    a.L = pan.L;
    a.amax = pan.amax;
    a.genotype = genotype;
    if (genotype) {
      a.n_items = nloc();
      a.item_base = i0;
      a.item_stride = pan.N;
    } else {
      a.n_items = H;
      a.item_base = 0;
      a.item_stride = H;
    }
    a.geno_lm = d_geno_lm.p;
    a.samp_lm = d_samp_lm.p;
    a.w = d_w.p;
    a.afreq = d_afreq.p;
    a.anum = d_anum.p;
    a.npos = d_npos.p;
    a.pos_allele = d_pos_allele.p;
    a.rank_of = d_rank_of.p;
    const long long w = wbase;  // global node index g lives at [g - wbase]
    a.parent = n_parent.p - w;
    a.start = n_start.p - w;
    a.allele = n_allele.p - w;
    a.flags = n_flags.p - w;
    a.freq = n_freq.p - w;
    a.prefix = n_prefix.p - w;
    a.tp = n_tp.p - w;
    a.sum = n_sum.p - w;
    a.cnt = n_cnt.p - w;
    a.size = n_size.p - w;
    a.pos = n_pos.p - w;
    a.child_base = n_child_base.p - w;
    a.link = n_link.p - w;
    a.list_off = n_list_off.p - w;
    a.region = n_region.p - w;
    a.r_region = d_r_region.p;
    a.r_child_base = d_r_child_base.p;
    a.rm = d_rm.p;
    return a;
  }

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
  int spell_table(const std::vector<int32_t> &ln, std::vector<int64_t> &off, std::vector<uint8_t> &al) {
    const int P = this->P;
    std::vector<int32_t> pp(P), node;
    std::vector<uint8_t> last(P);
    hipError_t e;
    if ((e = hipMemcpyAsync(pp.data(), t_ppat.p, (size_t)P * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(last.data(), t_last.p, (size_t)P, hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "table strings");
    off.assign((size_t)P + 1, 0);
    for (int i = 0; i < P; ++i) off[i + 1] = off[i] + ln[i];
    al.assign((size_t)off[P], 0);
    std::vector<int32_t> par;
    std::vector<uint8_t> alc;
    bool tree_loaded = false;
    for (int i = 0; i < P; ++i) {
      uint8_t *o = al.data() + off[i];
      o[ln[i] - 1] = last[i];
      const int32_t q = pp[i];
      if (ln[i] == 1) continue;
      if (q >= 0 && q < i && ln[q] == ln[i] - 1) {
        std::copy(al.data() + off[q], al.data() + off[q] + ln[q], o);
        continue;
      }
      if (!tree_ok()) return fail(HMC_EUNSUPPORTED, "allele strings of this table are unknown (a table set from outside)");
      if (!tree_loaded) {
        node.resize(P);
        if ((e = hipMemcpyAsync(node.data(), t_node.p, (size_t)P * 4, hipMemcpyDeviceToHost, st)) ||
            (e = hipStreamSynchronize(st)))
          return hipfail(e, "table strings");
        int nmax = 0;
        for (int k = 0; k < P; ++k) nmax = std::max(nmax, node[k] + 1);
        par.resize(nmax);
        alc.resize(nmax);
        if (nmax && ((e = hipMemcpyAsync(par.data(), n_parent.p, (size_t)nmax * 4, hipMemcpyDeviceToHost, st)) ||
                     (e = hipMemcpyAsync(alc.data(), n_allele.p, (size_t)nmax, hipMemcpyDeviceToHost, st)) ||
                     (e = hipStreamSynchronize(st))))
          return hipfail(e, "table strings");
        tree_loaded = true;
      }
      int32_t v = node[i];
      for (int k = ln[i] - 1; k >= 0; --k) {
        o[k] = alc[v];
        v = par[v];
      }
    }
    return HMC_OK;
  }

  // The current table with allele strings (mined: spelled from the prefix
  // ids; exact: the host copy).
  int table_to_host(Cands &c, std::vector<int32_t> &succ) {
    if (table_on_host) {
      c = ht;
      succ = ht_succ;
      return HMC_OK;
    }
    const int P = this->P, A = pan.amax;
    std::vector<int32_t> st(P), ln(P);
    std::vector<double> fr(P), pre(P), tp(P);
    std::vector<uint32_t> su((size_t)P * A);
    hipError_t e;
    if ((e = hipMemcpyAsync(st.data(), t_start.p, (size_t)P * 4, hipMemcpyDeviceToHost, this->st)) ||
        (e = hipMemcpyAsync(ln.data(), t_len.p, (size_t)P * 4, hipMemcpyDeviceToHost, this->st)) ||
        (e = hipMemcpyAsync(fr.data(), t_freq.p, (size_t)P * 8, hipMemcpyDeviceToHost, this->st)) ||
        (e = hipMemcpyAsync(pre.data(), t_prefix.p, (size_t)P * 8, hipMemcpyDeviceToHost, this->st)) ||
        (e = hipMemcpyAsync(tp.data(), t_tp.p, (size_t)P * 8, hipMemcpyDeviceToHost, this->st)) ||
        (e = hipMemcpyAsync(su.data(), t_succ.p, su.size() * 4, hipMemcpyDeviceToHost, this->st)) ||
        (e = hipStreamSynchronize(this->st)))
      return hipfail(e, "exact: table");
    std::vector<int64_t> off;
    std::vector<uint8_t> al;
    int rc = spell_table(ln, off, al);
    if (rc) return rc;
    c = Cands();
    for (int i = 0; i < P; ++i) c.push(st[i], ln[i], al.data() + off[i], 0, false, fr[i], pre[i], tp[i]);
    succ.resize((size_t)P * A);
    for (size_t i = 0; i < su.size(); ++i) succ[i] = su[i] == NONE ? -1 : (int32_t)su[i];
    return HMC_OK;
  }

  // One round: HaploBuilder::estimateFrequency(patterns) for c[b, e) —
  // ForwardPatternTree, then every individual of the shard through the
  // structure pass (forward links), exact_fb and exact_walk; fixed-point
  // sums over ranks; freq / prefix / tp as at HaploBuilder.cpp:317-331.
  int estimate_round(Cands &c, size_t b, size_t e) {
    const int L = pan.L, A = pan.amax, N = pan.N;
    const auto t_round = std::chrono::steady_clock::now();
    const double walk0 = ms_walk;
    const bool reused = xc_reuse;
    std::vector<int32_t> child, data, root(L, -1);
    int maxd = 0;
    auto new_node = [&]() {
      child.insert(child.end(), A, -1);
      data.push_back(-1);
      return (int32_t)data.size() - 1;
    };
    for (size_t k = b; k < e; ++k) {  // ForwardPatternTree::addPattern (PatternTree.cpp:188-212)
      const int s = c.start[k];
      if (root[s] < 0) root[s] = new_node();
      int32_t u = root[s];
      const uint8_t *al = c.alleles(k);
      for (int q = 0; q < c.len[k]; ++q) {
        if (al[q] >= A) return fail(HMC_EUNSUPPORTED, "exact M-step: pattern with a missing allele");
        int32_t v = child[(size_t)u * A + al[q]];
        if (v < 0) {
          v = new_node();
          child[(size_t)u * A + al[q]] = v;
        }
        u = v;
      }
      data[u] = (int32_t)(k - b);
      maxd = std::max(maxd, (int)c.len[k]);
    }
    const size_t nc = e - b;
    hipError_t er;
    if ((er = d_tr_child.ensure(std::max<size_t>(child.size(), 1))) || (er = d_tr_data.ensure(std::max<size_t>(data.size(), 1))) ||
        (er = d_tr_root.ensure(L)) || (er = d_xacc.ensure(2 * std::max<size_t>(nc, 1))) ||
        (!child.empty() && (er = hipMemcpyAsync(d_tr_child.p, child.data(), child.size() * 4, hipMemcpyHostToDevice, st))) ||
        (!data.empty() && (er = hipMemcpyAsync(d_tr_data.p, data.data(), data.size() * 4, hipMemcpyHostToDevice, st))) ||
        (er = hipMemcpyAsync(d_tr_root.p, root.data(), (size_t)L * 4, hipMemcpyHostToDevice, st)) ||
        (er = hipMemsetAsync(d_xacc.p, 0, 2 * nc * 8, st)))
      return hipfail(er, "exact: trie");
    tr_maxd = maxd;
    // the individuals of the shard, heaviest first, through the split machinery
    const int n = nloc();
    if ((er = d_xstatus.ensure(n)) || (er = d_xre.ensure(n)) || (er = d_xfmax.ensure(n))) return hipfail(er, "exact");
    std::vector<int32_t> order(n);
    for (int q = 0; q < n; ++q) order[q] = q;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return h_cost[x] > h_cost[y]; });
    xacc_nc = nc;
    int rc;
    if (xc_reuse) {
      if ((rc = exact_group(nullptr, xc_k))) return rc;
    } else {
      const int passes0 = n_struct_passes;
      while (true) {
        xc_groups = 0;
        rc = estep_split(order, true);
        if (rc != ESTEP_RESTART) break;
        if ((er = hipMemsetAsync(d_xacc.p, 0, 2 * nc * 8, st))) return hipfail(er, "exact");
      }
      if (rc) return rc;
      // one structure pass and one walk group: the stores hold every individual
      xc_reuse = n_struct_passes == passes0 + 1 && xc_groups == 1;
    }
    std::vector<unsigned long long> acc(2 * nc);
    if ((er = hipMemcpyAsync(acc.data(), d_xacc.p, acc.size() * 8, hipMemcpyDeviceToHost, st)) ||
        (er = hipStreamSynchronize(st)))
      return hipfail(er, "exact");
    if (multi()) {  // integer sums over ranks, exactly: 32-bit halves through the double collective
      std::vector<double> h(4 * nc);
      for (size_t i = 0; i < 2 * nc; ++i) {
        h[2 * i] = (double)(acc[i] & 0xFFFFFFFFull);
        h[2 * i + 1] = (double)(acc[i] >> 32);
      }
      if ((rc = allreduce_host(h.data(), h.size()))) return rc;
      for (size_t i = 0; i < 2 * nc; ++i) acc[i] = ((unsigned long long)h[2 * i + 1] << 32) + (unsigned long long)h[2 * i];
    }
    for (size_t k = 0; k < nc; ++k) {  // HaploBuilder.cpp:317-331
      double freq = std::min((double)acc[k] / EXACT_FIXED_SCALE, (double)N);
      const double pre = std::min((double)acc[nc + k] / EXACT_FIXED_SCALE, (double)N);
      freq = std::min(freq, pre);
      c.freq[b + k] = freq / N;
      c.prefix[b + k] = pre / N;
      const double t = pre > 0 ? freq / pre : freq / N;
      c.tp[b + k] = t < 1.0 ? t : 1.0;  // HaploPattern::setTransitionProb (HaploPattern.h:47)
    }
    ++exact_rounds;
    exact_candidates += nc;
    if (debug_mem)
      fprintf(stderr, "[hmc] exact round %d: %zu candidates, trie depth %d, walk %.1f ms, round %.1f ms%s\n", exact_rounds,
              nc, maxd, ms_walk - walk0,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_round).count(),
              reused ? " (E-step data reused)" : "");
    return HMC_OK;
  }
  size_t xacc_nc = 0;

  // exact_fb + exact_walk over the group d_order2[0, k) (structure records in place)
  int exact_group(const int32_t *ids, int k, const std::function<int(std::vector<int32_t> &)> &rerun = nullptr) {
    const int L = pan.L;
    int dev_cu = 256;
    hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
    hipError_t e;
    ExactArgs x;
    x.L = L;
    x.head_len = head_len;
    x.width = pan.amax;
    x.order = d_order2.p;
    x.n_order = k;
    x.rec = d_rec.p;
    x.rec_off = d_rec_off.p;
    x.status = d_xstatus.p;
    x.gprob = d_total.p;
    x.x = d_trace.p;
    x.x_base = d_tbase.p;
    x.x_off = d_loc_off.p;
    x.tr_child = d_tr_child.p;
    x.tr_data = d_tr_data.p;
    x.tr_root = d_tr_root.p;
    x.max_depth = tr_maxd;
    x.head_al = d_head_al.p;
    x.acc_freq = d_xacc.p;
    x.acc_prefix = d_xacc.p + xacc_nc;
    if (xc_reuse) {  // a later round over the same group: records and fwd/bwd sums are still in place
      x.fmax = xc_fmax;
      return exact_walk_group(x, k, dev_cu);
    }
    if ((e = launch_exact_fb(x, std::max(1, std::min(k, dev_cu * 8)), st))) return hipfail(e, "exact_fb");
    const int n = nloc();
    std::vector<int32_t> xs(n), fm(n);
    if ((e = hipMemcpyAsync(xs.data(), d_xstatus.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(fm.data(), d_xfmax.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "exact_fb");
    std::vector<int32_t> redo;
    for (int q = 0; q < k; ++q)
      if (xs[ids[q]] == EST_NEEDS_EXACT) redo.push_back(ids[q]);
    if (!redo.empty()) {  // their records again, pruned, then their fwd/bwd sums
      if (!rerun) return fail(HMC_EHIP, "exact M-step: a forward likelihood underflows (individual %d)", i0 + redo[0]);
      int rc;
      if ((rc = rerun(redo))) return rc;
      const int nr = (int)redo.size();
      if ((e = d_redo.ensure(nr))) return hipfail(e, "exact underflow re-run");
      if ((rc = upload_order(d_redo, redo.data(), nr))) return rc;
      ExactArgs x2 = x;
      x2.order = d_redo.p;
      x2.n_order = nr;
      if ((e = launch_exact_fb(x2, std::max(1, std::min(nr, dev_cu * 8)), st))) return hipfail(e, "exact_fb");
      if ((e = hipMemcpyAsync(xs.data(), d_xstatus.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(fm.data(), d_xfmax.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipStreamSynchronize(st)))
        return hipfail(e, "exact_fb");
      for (int r : redo)
        if (xs[r] == EST_NEEDS_EXACT) return fail(HMC_EHIP, "exact M-step: pruned records still underflow (individual %d)", i0 + r);
    }
    int fmax = 1;
    for (int q = 0; q < k; ++q) fmax = std::max(fmax, fm[ids[q]]);
    x.fmax = fmax;
    xc_fmax = fmax;
    xc_k = k;
    ++xc_groups;
    return exact_walk_group(x, k, dev_cu);
  }
  // The trie walk of one group (the current round's trie).
  int exact_walk_group(ExactArgs &x, int k, int dev_cu) {
    const int L = pan.L;
    hipError_t e;
    if (exact_walk_lds_bytes(tr_maxd, x.fmax) > EXACT_WALK_LDS_MAX)
      return fail(HMC_EUNSUPPORTED, "exact M-step: a frontier of %d states (trie depth %d) exceeds the walk's LDS bitmap",
                  x.fmax, tr_maxd);
    x.scratch_stride = exact_walk_scratch_doubles(tr_maxd, x.fmax, x.width);
    const long long items = (long long)k * L;
    // 28 waves per CU (7 per SIMD at 64 VGPRs), fewer when the per-wave lists
    // would pass SCRATCH_MAX
    const long long by_mem = std::max<long long>(1, (long long)(SCRATCH_MAX / (x.scratch_stride * 8)));
    const int grid = (int)std::max<long long>(1, std::min<long long>(std::min<long long>(items, (long long)dev_cu * 28), by_mem));
    // the walk's zero invariant (its lists; the child frequencies and touched
    // lists are left behind by each item and would land inside the lists of
    // a group whose depth or frontier differs): zeroed for every group
    const size_t need = x.scratch_stride * grid;
    if ((e = d_xscr.ensure(need)) || (e = hipMemsetAsync(d_xscr.p, 0, need * 8, st)))
      return hipfail(e, "exact scratch");
    x.scratch = d_xscr.p;
    // long walks (over 4 M items) in 16 slices, so that they report progress
    // (the lists return to zero between slices: every item clears its entries)
    const long long slice = items > (4ll << 20) ? std::max<long long>(grid, (items + 15) / 16) : items;
    for (long long i0 = 0; i0 < items; i0 += slice) {
      x.item0 = i0;
      x.item1 = std::min(items, i0 + slice);
      hipEventRecord(ev[0], st);
      if ((e = launch_exact_walk(x, grid, st))) return hipfail(e, "exact_walk");
      hipEventRecord(ev[1], st);
      if ((e = hipStreamSynchronize(st))) return hipfail(e, "exact_walk");
      float ms = 0;
      hipEventElapsedTime(&ms, ev[0], ev[1]);
      ms_walk += ms;
      if (debug_mem && items > 16 * (long long)grid)
        fprintf(stderr, "[hmc] exact walk: items %lld..%lld of %lld (%d individuals), %.1f ms\n", i0, x.item1, items, k, ms);
    }
    return HMC_OK;
  }
  double ms_walk = 0;
  // Rounds of one exact M-step share the E-step model: when a round's
  // individuals ran as one structure pass and one group, the next rounds walk
  // their new tries over the same records and fwd/bwd sums (exact_walk only).
  bool xc_reuse = false;
  int xc_groups = 0, xc_fmax = 1, xc_k = 0;

  // Successors of a pattern set (PatternManager::initialize, :308-317):
  // successor[j] = the longest stored suffix of (pattern + allele j) with start
  // >= the pattern's start; found through a trie of the set per start locus.
  void host_successors(const Cands &c, std::vector<int32_t> &succ) {
    const int L = pan.L, A = pan.amax;
    const size_t P = c.size();
    std::vector<int32_t> child, data, root(L, -1);
    auto new_node = [&]() {
      child.insert(child.end(), A, -1);
      data.push_back(-1);
      return (int32_t)data.size() - 1;
    };
    for (size_t k = 0; k < P; ++k) {
      const int s = c.start[k];
      if (root[s] < 0) root[s] = new_node();
      int32_t u = root[s];
      const uint8_t *al = c.alleles(k);
      for (int q = 0; q < c.len[k]; ++q) {
        int32_t v = child[(size_t)u * A + al[q]];
        if (v < 0) {
          v = new_node();
          child[(size_t)u * A + al[q]] = v;
        }
        u = v;
      }
      data[u] = (int32_t)k;
    }
    succ.assign(P * A, -1);
    for (size_t k = 0; k < P; ++k) {
      const int s = c.start[k], ln = c.len[k], e = s + ln;
      if (e >= L) continue;
      const uint8_t *al = c.alleles(k);
      for (int j = 0; j < h_anum[e]; ++j) {
        int32_t res = -1;
        for (int s2 = s; s2 <= e && res < 0; ++s2) {  // longest first
          int32_t u = root[s2];
          for (int q = s2 - s; q < ln && u >= 0; ++q) u = child[(size_t)u * A + al[q]];
          if (u >= 0) u = child[(size_t)u * A + j];
          if (u >= 0) res = data[u];
        }
        succ[k * A + j] = res;
      }
    }
  }

  // Install a host-built table (id order) on the device: SoA, successors,
  // heads (PatternManager.cpp:293-318).
  int install_host_table(Cands &c, std::vector<int32_t> &succ) {
    const int P = (int)c.size(), A = pan.amax;
    if ((int64_t)P > INT32_MAX) return fail(HMC_EUNSUPPORTED, "too many patterns");
    int rc = alloc_table(std::max(P, 1));
    if (rc) return rc;
    std::vector<uint8_t> last(P);
    std::vector<int32_t> node(P, -1);
    std::vector<uint32_t> su((size_t)P * A);
    for (int i = 0; i < P; ++i) last[i] = c.alleles(i)[c.len[i] - 1];
    for (size_t i = 0; i < su.size(); ++i) su[i] = succ[i] < 0 ? NONE : (uint32_t)succ[i];
    hipError_t e;
    if (P && ((e = hipMemcpyAsync(t_start.p, c.start.data(), (size_t)P * 4, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_len.p, c.len.data(), (size_t)P * 4, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_node.p, node.data(), (size_t)P * 4, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_freq.p, c.freq.data(), (size_t)P * 8, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_prefix.p, c.prefix.data(), (size_t)P * 8, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_tp.p, c.tp.data(), (size_t)P * 8, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_last.p, last.data(), (size_t)P, hipMemcpyHostToDevice, st)) ||
              (e = hipMemcpyAsync(t_succ.p, su.data(), su.size() * 4, hipMemcpyHostToDevice, st)) ||
              (e = hipMemsetAsync(t_ppat.p, 0xFE, (size_t)P * 4, st)) ||  // alleles are kept on the host (ht)
              (e = hipStreamSynchronize(st))))
      return hipfail(e, "exact: install table");
    this->P = P;
    // head list: start 0, length head_len, id order (PatternManager.cpp:304-306)
    std::vector<std::pair<uint32_t, uint8_t>> heads;
    h_head_ids.clear();
    h_head_al.clear();
    std::vector<uint8_t> tab;
    if (head_len > 1) tab.assign((size_t)std::max(P, 1) * head_len, 0);
    for (int i = 0; i < P; ++i)
      if (c.start[i] == 0 && c.len[i] == head_len) {
        heads.push_back({(uint32_t)i, c.alleles(i)[head_len - 1]});
        if (head_len > 1) {
          h_head_ids.push_back((uint32_t)i);
          h_head_al.insert(h_head_al.end(), c.alleles(i), c.alleles(i) + head_len);
          std::copy(c.alleles(i), c.alleles(i) + head_len, tab.begin() + (size_t)i * head_len);
        }
      }
    if (head_len > 1 && ((e = d_head_al.ensure(tab.size())) ||
                         (e = hipMemcpyAsync(d_head_al.p, tab.data(), tab.size(), hipMemcpyHostToDevice, st)) ||
                         (e = hipStreamSynchronize(st))))
      return hipfail(e, "exact: heads");
    if ((rc = set_heads(heads))) return rc;
    ht = c;
    ht_succ = succ;
    table_on_host = true;
    have_model = true;
    new_table(false);
    return HMC_OK;
  }

  // PatternManager::estimatePatterns (PatternManager.cpp:364-410).
  int estimate_patterns(int *P_out, uint64_t *rm_out) {
    if (!have_estep) return fail(HMC_EARG, "exact M-step needs an E-step first");
    // after findPatternByNum the reference estimates at that search's last
    // threshold (m_min_freq, PatternManager.cpp:53-60, 364-408)
    const bool bynum = num_patterns > 0 && model != 1;
    if (bynum && !(bynum_theta_last > 0))
      return fail(HMC_EARG, "exact M-step after findPatternByNum needs the search's threshold (mine first)");
    if (pan.amax > 44)  // the records pack a locus's allele pairs (amax (amax + 1) / 2) in 10 bits
      return fail(HMC_EUNSUPPORTED, "exact M-step with more than 44 alleles per locus");
    hipEventRecord(ev[4], st);
    const int L = pan.L;
    int mxl = max_len <= 0 ? L : max_len;  // m_max_len / m_min_len of the last findPatternByFreq
    int mnl = std::max(min_len, 1);
    mxl = std::max(mxl, mnl);
    double mf = bynum ? bynum_theta_last : current_min_freq();
    if (model == 1) {  // findPatternBlock: m_min_freq = -1 (PatternManager.cpp:75-88)
      mnl = mxl = std::max(1, mc_order + 1);
      mf = -1.0;
    }
    exact_rounds = 0;
    exact_candidates = 0;
    ms_walk = 0;
    xc_reuse = false;
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    auto t0 = clk::now();
    Cands cur;
    std::vector<int32_t> succ;
    int rc = table_to_host(cur, succ);
    if (rc) return rc;
    const double ms_to_host = ms_since(t0);
    t0 = clk::now();
    const int A = pan.amax;
    if (mf < 0) {  // estimateFrequency() (:347-362): re-estimate in place, ids and successors unchanged
      if ((rc = estimate_round(cur, 0, cur.size()))) return rc;
      if ((rc = install_host_table(cur, succ))) return rc;
    } else {
      Cands all;
      std::vector<size_t> seeds;
      for (size_t i = 0; i < cur.size(); ++i) {
        all.push(cur.start[i], cur.len[i], cur.alleles(i), 0, false, cur.freq[i], cur.prefix[i], cur.tp[i]);
        const int s = cur.start[i], e = s + cur.len[i];
        if (e < L && cur.len[i] < mxl)
          for (int j = 0; j < h_anum[e]; ++j) {
            const int32_t sj = succ[i * A + j];
            if (sj < 0 || cur.start[sj] != s) {  // the extension is not stored: a seed
              all.push(s, cur.len[i] + 1, cur.alleles(i), (uint8_t)j, true, cur.freq[i]);
              seeds.push_back(all.size() - 1);
            }
          }
      }
      size_t rb = 0, re = all.size();
      std::vector<uint8_t> buf;
      while (rb < re) {
        if ((rc = estimate_round(all, rb, re))) return rc;
        const size_t nb = all.size();
        for (int level = 0; level < 4; ++level) {  // extendPatterns (:412-438)
          std::vector<size_t> ns;
          for (size_t si : seeds) {
            const int s = all.start[si], ln = all.len[si], e = s + ln;
            if (e < L && ln < mxl && all.freq[si] >= mf) {
              buf.assign(all.alleles(si), all.alleles(si) + ln);
              const double f = all.freq[si];
              for (int j = 0; j < h_anum[e]; ++j) {
                all.push(s, ln + 1, buf.data(), (uint8_t)j, true, f);
                ns.push_back(all.size() - 1);
              }
            }
          }
          seeds.swap(ns);
        }
        rb = nb;
        re = all.size();
      }
      const double ms_rounds = ms_since(t0);
      t0 = clk::now();
      Cands kept;  // (:396-408)
      for (size_t i = 0; i < all.size(); ++i)
        if (all.freq[i] >= mf || all.len[i] <= mnl)
          kept.push(all.start[i], all.len[i], all.alleles(i), 0, false, all.freq[i], all.prefix[i], all.tp[i]);
      std::vector<int32_t> ksucc;
      host_successors(kept, ksucc);
      const double ms_succ = ms_since(t0);
      t0 = clk::now();
      if ((rc = install_host_table(kept, ksucc))) return rc;
      if (debug_mem)
        fprintf(stderr, "[hmc] exact M-step: table to host %.1f ms, rounds %.1f ms (walks %.1f), kept + successors %.1f ms, "
                "install %.1f ms\n", ms_to_host, ms_rounds, ms_walk, ms_succ, ms_since(t0));
    }
    xc_reuse = false;
    hipEventRecord(ev[5], st);
    hipError_t e;
    if ((e = hipStreamSynchronize(st))) return hipfail(e, "exact");
    // the walk's scratch (up to SCRATCH_MAX) and the tries go back to the E-step
    d_xscr.release();
    d_tr_child.release();
    d_tr_data.release();
    float ms = 0;
    hipEventElapsedTime(&ms, ev[4], ev[5]);
    ms_m = ms;
    if (P_out) *P_out = P;
    if (rm_out) *rm_out = 0;  // no candidate x item scans: the cost is in the trie walks
    return HMC_OK;
  }

  int mine(int *P_out, uint64_t *rm_out) {
    // HaploModel.cpp:140-144: after an E-step, --exact-estimate re-estimates
    // (estimatePatterns) instead of re-mining the samples
    if (exact_estimate && have_samples && have_model) return estimate_patterns(P_out, rm_out);
    table_on_host = false;
    if (!(num_patterns > 0 && model != 1)) return mine_impl(P_out, rm_out, 0);
    int k = 8;
    while (true) {
      const int rc = mine_impl(P_out, rm_out, k);
      if (rc != MINE_RETRY) return rc;
      k = std::max(bynum_need, 2 * k);
    }
  }
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
  int mine_impl_body(int *P_out, uint64_t *rm_out, int bynum_rounds) {
    if (!have_panel) return fail(HMC_EARG, "no panel loaded");
    const int L = pan.L;
    hipError_t e;
    hipEventRecord(ev[4], st);
    // PatternManager::findPatternByFreq argument normalisation (PatternManager.cpp:29-32)
    int mxl = max_len <= 0 ? L : max_len;
    int mnl = std::max(min_len, 1);
    mxl = std::max(mxl, mnl);
    double mf = current_min_freq();
    if (model == 1) {  // MC: findPatternBlock(mc_order+1) (PatternManager.cpp:72-88)
      mnl = mxl = std::max(1, mc_order + 1);
      mf = -1.0;
    }
    if (bynum_rounds > 0) mf = bynum_theta(bynum_rounds);
    if ((e = d_rm.ensure(RM_SLOTS * 16)) || (e = d_totals.ensure(2)) || (e = h_totals.ensure(2)) ||
        (e = d_rsize.ensure(L)) || (e = d_rpos.ensure(L)) || (e = d_r_region.ensure(L)) ||
        (e = hipMemsetAsync(d_rm.p, 0, RM_SLOTS * 16 * 8, st)))
      return hipfail(e, "mine");
    int W = block_width(L, mxl, mnl, bynum_rounds);
    if ((e = d_mine_err.ensure(1)) || (e = hipMemsetAsync(d_mine_err.p, 0, 4, st))) return hipfail(e, "mine");
    wbase = 0;
    long long next_node = 0;  // global index of the next node
    long long id_base = 0;    // patterns of the blocks above
    uint64_t rm_bynum = 0;
    int rc, nblocks = 0;
    mine_touched = true;
    for (int hi = L; hi > 0;) {
      const int lo = std::max(0, hi - W);
      MineBlock mb;
      if ((e = d_rm_save.ensure(RM_SLOTS * 16)) ||
          (e = hipMemcpyAsync(d_rm_save.p, d_rm.p, RM_SLOTS * 16 * 8, hipMemcpyDeviceToDevice, st)))
        return hipfail(e, "mine");
      rc = mine_block(lo, hi, mxl, mnl, mf, bynum_rounds, next_node, id_base, mb, rm_bynum);
      if (rc == MINE_SPLIT) {  // nothing of the block is kept: its R_M counts go, its nodes are overwritten
        if (bynum_rounds > 0 || mnl > 1 || hi - lo <= 1)
          return fail(HMC_ENOMEM, "pattern search: out of device memory (blocks of %d start loci)", hi - lo);
        if ((e = hipMemcpyAsync(d_rm.p, d_rm_save.p, RM_SLOTS * 16 * 8, hipMemcpyDeviceToDevice, st)))
          return hipfail(e, "mine");
        W = std::max(1, (hi - lo + 1) / 2);
        if (debug_mem) fprintf(stderr, "[hmc] mine block [%d, %d): out of memory, %d start loci per block from here\n", lo, hi, W);
        continue;
      }
      if (rc) return rc;
      // the block above this one is no longer needed
      if ((rc = slide_window(mb.first_node, mb.end_node))) return rc;
      next_node = mb.end_node;
      id_base += mb.patterns;
      ++nblocks;
      if (debug_mem && W < L)
        fprintf(stderr, "[hmc] mine block %d: start loci [%d, %d), %lld patterns so far, node window %lld..%lld\n",
                nblocks, lo, hi, id_base, (long long)mb.first_node, (long long)mb.end_node);
      hi = lo;
    }
    {  // before anything is committed: a failed successor walk leaves no table
      int merr = 0;
      if ((e = hipMemcpyAsync(&merr, d_mine_err.p, 4, hipMemcpyDeviceToHost, st)) || (e = hipStreamSynchronize(st)))
        return hipfail(e, "mine");
      if (merr) return fail(HMC_EUNSUPPORTED, "successor walk left the node window (blocks of %d start loci)", W);
    }
    tree_complete = nblocks == 1;
    P = (int)id_base;
    if (!tree_complete) {  // a partial tree is of no further use (strings come from ppat): give its memory back
      n_parent.release(); n_start.release(); n_child_base.release(); n_link.release(); n_allele.release();
      n_flags.release(); n_freq.release(); n_prefix.release(); n_tp.release(); n_sum.release(); n_cnt.release();
      n_size.release(); n_pos.release(); n_list_off.release(); n_region.release();
      last_mine_window_gb = (double)node_cap * 70.0 / 1e9;
      node_cap = 0;
      wbase = 0;
    } else {
      last_mine_window_gb = (double)node_cap * 70.0 / 1e9;
    }
    std::vector<unsigned long long> rm_slots((size_t)RM_SLOTS * 16);
    if ((e = hipMemcpyAsync(rm_slots.data(), d_rm.p, rm_slots.size() * 8, hipMemcpyDeviceToHost, st)))
      return hipfail(e, "mine");
    hipEventRecord(ev[5], st);
    if ((e = hipStreamSynchronize(st))) return hipfail(e, "mine");
    // The matching lists of the genotype branch (M0) reach tens of GB at
    // cfg 3 (R_M ~ 10^11 entries); give them back to the E-step's stores.
    for (int k = 0; k < 2; ++k) {
      if (l_idx[k].n * 4 > (4ull << 30)) l_idx[k].release();
      if (l_val[k].n * 8 > (4ull << 30)) l_val[k].release();
    }
    if (debug_mem) {
      size_t fb = 0, tb = 0;
      hipMemGetInfo(&fb, &tb);
      fprintf(stderr, "[hmc] after mining: %d patterns in %d block(s) of %d start loci, %lld nodes; free %.1f GB of %.1f; "
              "node window %.1f GB\n", P, nblocks, W, next_node, fb / 1e9, tb / 1e9, last_mine_window_gb);
    }
    unsigned long long rm = 0;
    for (int k = 0; k < RM_SLOTS; ++k) rm += rm_slots[(size_t)k * 16];
    if (bynum_rounds > 0) rm = rm_bynum;  // the scans of the candidates the rounds generated
    float ms = 0;
    hipEventElapsedTime(&ms, ev[4], ev[5]);
    ms_m = ms;
    have_model = true;
    new_table(true);
    last_mine_blocks = nblocks;
    last_mine_nodes = next_node;
    if (P_out) *P_out = P;
    if (rm_out) *rm_out = rm;
    return HMC_OK;
  }
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
                 MineBlock &mb, uint64_t &rm_bynum) {
    const bool genotype = !have_samples;
    const int L = pan.L;
    hipError_t e;
    int rc;
    std::vector<long long> lbeg{0, 0}, lend{0, 0};  // per level node ranges (index = level), global
    long long n1 = 0;
    for (int k = lo; k < hi; ++k) n1 += h_npos[k];
    // Out of device memory for the block's nodes or lists: the block is
    // re-run with half the width (mine_impl).  Ranks agree on it (one flag
    // all-reduced per level), so that all of them split the same block.
    auto oom_split = [&](int rc_in, bool oom) -> int {
      if (multi()) {
        double f = oom ? 1.0 : 0.0;
        hipError_t e2;
        if ((e2 = d_flag.ensure(1)) || (e2 = hipMemcpyAsync(d_flag.p, &f, 8, hipMemcpyHostToDevice, st)))
          return hipfail(e2, "mine");
        if (int r2 = allreduce_sum(d_flag.p, 1)) return r2;
        if ((e2 = hipMemcpyAsync(&f, d_flag.p, 8, hipMemcpyDeviceToHost, st)) || (e2 = hipStreamSynchronize(st)))
          return hipfail(e2, "mine");
        oom = f > 0.0;
      }
      if (oom) {
        (void)hipGetLastError();
        return MINE_SPLIT;
      }
      return rc_in;
    };
    nodes_oom = false;
    rc = grow_nodes((size_t)std::max<long long>(node0 + n1, 1), (size_t)node0);
    if ((rc = oom_split(rc, rc && nodes_oom))) return rc;
    if (node0 + n1 > (long long)INT32_MAX) return fail(HMC_EUNSUPPORTED, "candidate tree exceeds 2^31 nodes");
    // level-1 nodes of the block's roots (r_child_base of root k) and the
    // roots' child lists: root r owns npos[r] x n_items slots of the next buffer
    unsigned long long next_total = 0;
    {
      const unsigned long long ni = (unsigned long long)mine_args(genotype).n_items;
      std::vector<unsigned long long> rr(hi - lo);
      std::vector<int32_t> rcb(hi - lo);
      long long c = node0;
      for (int k = lo; k < hi; ++k) {
        rr[k - lo] = next_total;
        next_total += (unsigned long long)h_npos[k] * ni;
        rcb[k - lo] = (int32_t)c;
        c += h_npos[k];
      }
      if ((e = hipMemcpyAsync(d_r_region.p + lo, rr.data(), rr.size() * 8, hipMemcpyHostToDevice, st)) ||
          (e = hipMemcpyAsync(d_r_child_base.p + lo, rcb.data(), rcb.size() * 4, hipMemcpyHostToDevice, st)))
        return hipfail(e, "mine");
    }
    lbeg[1] = node0;
    lend[1] = node0 + n1;
    int level = 1;
    long long pbeg = lo, pend = hi;  // level-1 parents are the block's roots
    int cur = 0;                     // list buffer holding the parents' lists
    while (true) {
      const long long cb = lbeg[level], ce = lend[level];
      const int nlev = (int)(ce - cb);
      const int nxt = cur ^ 1;  // children's lists are written here during the count
      const unsigned long long list_bytes = next_total * (genotype ? 12ull : 4ull);
      if (mine_list_cap && list_bytes > mine_list_cap) {
        if ((rc = oom_split(HMC_OK, true))) return rc;
      }
      e = ensure_or_release(l_idx[nxt], std::max<unsigned long long>(next_total, 1));
      if (!e && genotype) e = ensure_or_release(l_val[nxt], std::max<unsigned long long>(next_total, 1));
      if ((rc = oom_split(e ? hipfail(e, "mine lists") : HMC_OK, e == hipErrorOutOfMemory))) return rc;
      MineArgs a = mine_args(genotype);
      a.lout_idx = l_idx[nxt].p;
      a.lout_val = genotype ? l_val[nxt].p : nullptr;
      a.denom = genotype ? (double)pan.N : total_weight;
      a.min_freq = mf;
      a.min_len = mnl;
      a.max_len = mxl;
      a.lin_idx = level == 1 ? nullptr : l_idx[cur].p;
      a.lin_val = level == 1 ? nullptr : l_val[cur].p;
      hipEvent_t dm0 = nullptr, dm1 = nullptr;
      if (diag_mine) {
        hipEventCreate(&dm0);
        hipEventCreate(&dm1);
        hipEventRecord(dm0, st);
      }
#ifdef HMC_STAMPS
      if (diag_mine) {
        d_mstamps.ensure((size_t)(pend - pbeg) * 8);
        hipMemsetAsync(d_mstamps.p, 0, (size_t)(pend - pbeg) * 64, st);
        a.stamps = d_mstamps.p;
      }
#endif
      if (multi() && reduction == RED_ORDERED) {
        // every rank scans its items and writes the children's lists at once;
        // then rank r continues every child's sum from ranks 0..r-1 (items in
        // order) over its lists and passes it on
        if ((e = launch_mine_count(a, level, (int)pbeg, (int)pend, st))) return hipfail(e, "mine_count");
        for (int r = 0; r < world; ++r) {
          if (r == rank && r > 0 && (e = launch_mine_sum(a, (int)cb, (int)ce, st))) return hipfail(e, "mine_sum");
          if ((rc = bcast(n_sum.p + (cb - wbase), nlev, r))) return rc;
        }
      } else if ((e = launch_mine_count(a, level, (int)pbeg, (int)pend, st))) {
        return hipfail(e, "mine_count");
      }
      if (diag_mine) {  // per-level list statistics of the parents (diagnostic)
        hipEventRecord(dm1, st);
        hipStreamSynchronize(st);
        float ms = 0;
        hipEventElapsedTime(&ms, dm0, dm1);
        size_t tot_n = 0, max_n = 0, npar = 0;
        if (level == 1) {
          npar = (size_t)(hi - lo);
          tot_n = npar * (size_t)a.n_items;
          max_n = (size_t)a.n_items;
        } else {
          std::vector<uint32_t> hc((size_t)(pend - pbeg));
          std::vector<uint8_t> hf((size_t)(pend - pbeg));
          hipMemcpy(hc.data(), n_cnt.p + (pbeg - wbase), hc.size() * 4, hipMemcpyDeviceToHost);
          hipMemcpy(hf.data(), n_flags.p + (pbeg - wbase), hf.size(), hipMemcpyDeviceToHost);
          for (size_t q = 0; q < hc.size(); ++q)
            if (hf[q] & 2) {
              ++npar;
              tot_n += hc[q];
              max_n = std::max<size_t>(max_n, hc[q]);
            }
        }
        fprintf(stderr, "mine block [%d,%d) level %2d: %7zu ext parents of %7lld, entries %9zu, max list %7zu, "
                "mine_count %.3f ms\n", lo, hi, level, npar, pend - pbeg, tot_n, max_n, ms);
#ifdef HMC_STAMPS
        unsigned long long hs[8] = {};
        std::vector<unsigned long long> hv((size_t)(pend - pbeg) * 8);
        hipMemcpy(hv.data(), d_mstamps.p, hv.size() * 8, hipMemcpyDeviceToHost);
        for (size_t q = 0; q < hv.size(); ++q) hs[q % 8] += hv[q];
        const double nwv = hs[5] ? (double)hs[5] : 1.0;
        fprintf(stderr, "   per wave (cycles): view %.0f  loads %.0f  compact %.0f  sum %.0f  epilogue %.0f; waves %llu\n",
                hs[0] / nwv, hs[1] / nwv, hs[2] / nwv, hs[3] / nwv, hs[4] / nwv, hs[5]);
#endif
        hipEventDestroy(dm0);
        hipEventDestroy(dm1);
      }
      if (!(multi() && reduction == RED_ORDERED) && (rc = allreduce_sum(n_sum.p + (cb - wbase), nlev))) return rc;
      if ((e = s_ext.ensure(nlev)) || (e = s_child.ensure(nlev))) return hipfail(e, "mine");
      const size_t tmpb = mine_scan_tmp_bytes(nlev);
      if ((e = s_tmp.ensure(tmpb))) return hipfail(e, "mine");
      if ((e = launch_mine_finalize(a, level, (int)cb, (int)ce, s_ext.p, s_child.p, st))) return hipfail(e, "mine_finalize");
      if ((e = launch_mine_offsets(a, (int)cb, (int)ce, s_ext.p, s_child.p, (int)ce, s_tmp.p, s_tmp.n, d_totals.p, st)))
        return hipfail(e, "mine_offsets");
      const unsigned long long *tot = h_totals.p;
      if ((e = hipMemcpyAsync(h_totals.p, d_totals.p, 16, hipMemcpyDeviceToHost, st)) || (e = hipStreamSynchronize(st)))
        return hipfail(e, "mine");
      next_total = tot[0];  // list slots the next level's children need
      if (tot[1] > (unsigned long long)INT32_MAX - (unsigned long long)ce)
        return fail(HMC_EUNSUPPORTED, "candidate tree exceeds 2^31 nodes at length %d", level + 1);
      const long long nnext = (long long)tot[1];
      cur = nxt;
      if (nnext == 0) break;
      pbeg = cb;
      pend = ce;
      ++level;
      lbeg.push_back(ce);
      lend.push_back(ce + nnext);
      nodes_oom = false;
      rc = grow_nodes((size_t)(ce + nnext), (size_t)ce);
      if ((rc = oom_split(rc, rc && nodes_oom))) return rc;
    }
    const int maxlev = level;
    MineArgs a = mine_args(genotype);
    long long Pb = 0;
    if (bynum_rounds > 0) {  // one block: the node window starts at 0
      rc = bynum_replay(a, (int)lend[maxlev], mnl, mxl, bynum_rounds, rm_bynum);
      if (rc) return rc;
      Pb = P;
    } else {
      // DFS pre-order ids from subtree sizes
      for (int lv = maxlev; lv >= 1; --lv)
        if ((e = launch_mine_size(a, lv, (int)lbeg[lv], (int)lend[lv], st))) return hipfail(e, "mine_size");
      if ((e = launch_mine_root_size(a, d_rsize.p, lo, hi, st))) return hipfail(e, "mine_root_size");
      std::vector<uint32_t> rsize(hi - lo), rpos(hi - lo);
      if ((e = hipMemcpyAsync(rsize.data(), d_rsize.p + lo, rsize.size() * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipStreamSynchronize(st)))
        return hipfail(e, "mine");
      uint64_t acc = (uint64_t)id_base;
      for (int s = hi - 1; s >= lo; --s) {  // roots popped from the back: start L-1 first
        rpos[s - lo] = (uint32_t)acc;
        acc += rsize[s - lo];
      }
      if (acc > (uint64_t)INT32_MAX) return fail(HMC_EUNSUPPORTED, "too many patterns (%llu)", (unsigned long long)acc);
      Pb = (long long)acc - id_base;
      if ((e = hipMemcpyAsync(d_rpos.p + lo, rpos.data(), rpos.size() * 4, hipMemcpyHostToDevice, st)))
        return hipfail(e, "mine");
      if ((e = launch_mine_pos(a, 1, lo, hi, d_rpos.p, st))) return hipfail(e, "mine_pos");
      for (int lv = 2; lv <= maxlev; ++lv)
        if ((e = launch_mine_pos(a, lv, (int)lbeg[lv - 1], (int)lend[lv - 1], d_rpos.p, st))) return hipfail(e, "mine_pos");
    }
    if ((rc = grow_table((size_t)(id_base + Pb), (size_t)id_base))) return rc;
    PatternTable t = table();
    std::vector<int> lb(maxlev + 2);  // the block's level ranges (global node indices < 2^31)
    for (int lv = 1; lv <= maxlev; ++lv) lb[lv] = (int)lbeg[lv];
    lb[maxlev + 1] = (int)lend[maxlev];
    if ((e = d_lev_begin.ensure(lb.size())) ||
        (e = hipMemcpyAsync(d_lev_begin.p, lb.data(), lb.size() * 4, hipMemcpyHostToDevice, st)) ||
        (e = launch_mine_emit(a, d_lev_begin.p, maxlev, lb[maxlev + 1] - lb[1], t, st)))
      return hipfail(e, "mine_emit");
    for (int lv = 1; lv <= maxlev; ++lv)
      if ((e = launch_mine_succ_level(a, t, lv, (int)lbeg[lv], (int)lend[lv], (int32_t)wbase, d_mine_err.p, st)))
        return hipfail(e, "mine_succ");
    if (lo == 0) {
      head_len = mnl;
      P = (int)(id_base + Pb);  // the head pairs' lookups see the whole table
      if ((rc = build_heads_from_nodes(a, mnl <= maxlev ? (int)lbeg[mnl] : 0, mnl <= maxlev ? (int)lend[mnl] : 0))) return rc;
    }
    mb.first_node = node0;
    mb.end_node = lend[maxlev];
    mb.patterns = Pb;
    return HMC_OK;
  }

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
  int grow_table(size_t n, size_t used) {
    hipError_t e;
    n = std::max<size_t>(n, 1);
    const size_t A = (size_t)pan.amax;
    auto grow = [&]() -> hipError_t {
      hipError_t r;
      if ((r = t_start.grow_keep(n, used, st)) || (r = t_len.grow_keep(n, used, st)) ||
          (r = t_node.grow_keep(n, used, st)) || (r = t_freq.grow_keep(n, used, st)) ||
          (r = t_prefix.grow_keep(n, used, st)) || (r = t_tp.grow_keep(n, used, st)) ||
          (r = t_last.grow_keep(n, used, st)) || (r = t_ppat.grow_keep(n, used, st)) ||
          (r = t_succ.grow_keep(n * A, used * A, st)))
        return r;
      return hipSuccess;
    };
    if ((e = grow()) == hipErrorOutOfMemory) {
      // the table grows after a block's search: its matching lists (sized by
      // the block's largest level) and the E-step stores can go
      (void)hipGetLastError();
      for (int k = 0; k < 2; ++k) {
        l_idx[k].release();
        l_val[k].release();
      }
      d_trace.release();
      d_rec.release();
      e = grow();
    }
    if (e) return hipfail(e, "grow_table");
    return HMC_OK;
  }
  PatternTable table() const {
    PatternTable t;
    t.start = t_start.p;
    t.len = t_len.p;
    t.node = t_node.p;
    t.ppat = t_ppat.p;
    t.freq = t_freq.p;
    t.prefix = t_prefix.p;
    t.tp = t_tp.p;
    t.last = t_last.p;
    t.succ = t_succ.p;
    return t;
  }

  // Head list (PatternManager.cpp:304-306) and the locus-0 lookup used by
  // initHeadList's findLongestMatchPattern(head_len, ...) for head_len == 1.
  int set_heads(const std::vector<std::pair<uint32_t, uint8_t>> &heads /* (id, allele at 0) */) {
    std::vector<uint32_t> ids, pat0(pan.amax + 1, NONE);
    for (auto &h : heads) {
      ids.push_back(h.first);
      pat0[h.second] = h.first;
    }
    std::sort(ids.begin(), ids.end());
    for (int x = 0; x < pan.amax; ++x)
      if (pat0[x] != NONE) { pat0[pan.amax] = pat0[x]; break; }
    n_head = (int)ids.size();
    hipError_t e;
    if ((e = d_head_ids.ensure(std::max<size_t>(ids.size(), 1))) || (e = d_head_pat0.ensure(pat0.size())))
      return hipfail(e, "set_heads");
    if (!ids.empty() &&
        (e = hipMemcpyAsync(d_head_ids.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, st)))
      return hipfail(e, "set_heads");
    if ((e = hipMemcpyAsync(d_head_pat0.p, pat0.data(), pat0.size() * 4, hipMemcpyHostToDevice, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "set_heads");
    return HMC_OK;
  }

  // The rounds of findPatternByNum over the candidate tree mined at
  // theta(rounds): acceptance order, the last round sorted by frequency
  // (std::sort, HaploPattern::greater_frequency) and cut; then node flags and
  // positions so that mine_emit / mine_succ build the table in that order.
  int bynum_replay(const MineArgs &, int ntot, int mnl, int mxl, int, uint64_t &rm_out) {
    const int L = pan.L;
    hipError_t e;
    std::vector<uint8_t> fl(ntot);
    std::vector<int32_t> cb(ntot), stt(ntot);
    std::vector<double> fr(ntot);
    std::vector<uint32_t> cnt(ntot);
    if (ntot > 0 &&
        ((e = hipMemcpyAsync(fl.data(), n_flags.p, (size_t)ntot, hipMemcpyDeviceToHost, st)) ||
         (e = hipMemcpyAsync(cb.data(), n_child_base.p, (size_t)ntot * 4, hipMemcpyDeviceToHost, st)) ||
         (e = hipMemcpyAsync(stt.data(), n_start.p, (size_t)ntot * 4, hipMemcpyDeviceToHost, st)) ||
         (e = hipMemcpyAsync(fr.data(), n_freq.p, (size_t)ntot * 8, hipMemcpyDeviceToHost, st)) ||
         (e = hipMemcpyAsync(cnt.data(), n_cnt.p, (size_t)ntot * 4, hipMemcpyDeviceToHost, st)) ||
         (e = hipStreamSynchronize(st))))
      return hipfail(e, "bynum");
    const unsigned long long n_items = (unsigned long long)mine_args(!have_samples).n_items;
    struct C { int32_t v; int len; };  // v < 0: root of start -v-1 (the empty pattern)
    std::vector<C> stack, kept;
    std::vector<int32_t> out;
    for (int s0 = 0; s0 < L; ++s0) stack.push_back({-(s0 + 1), 0});  // generateCandidates
    uint64_t rm = 0;
    double theta = 1.0;
    int max_num = num_patterns, last_size = 0;
    // searchPattern(true) at threshold theta (PatternManager.cpp:100-144)
    auto search = [&](int round) -> int {
      kept.clear();
      while (!stack.empty()) {
        const C c = stack.back();
        stack.pop_back();
        const bool root = c.v < 0;
        const int start = root ? -c.v - 1 : stt[c.v];
        const double f = root ? 1.0 : fr[c.v];  // the empty pattern has frequency 1
        const int end = start + c.len;
        if (f >= theta || c.len < mnl) {
          if (end < L && c.len < mxl) {
            if (!root && !(fl[c.v] & NODE_EXT)) return round;  // the mined tree is too shallow
            const int base = root ? [&] { int b = 0; for (int k = 0; k < start; ++k) b += h_npos[k]; return b; }()
                                  : cb[c.v];
            const unsigned long long scan = root ? n_items : (cnt[c.v] > 0 ? cnt[c.v] : n_items);
            for (int j = 0; j < h_npos[end]; ++j) {
              stack.push_back({base + j, c.len + 1});
              rm += scan;  // checkFrequencyWithExtension of the new candidate
            }
          }
        }
        if (f >= theta || c.len <= mnl) {
          if (c.len > 0 && c.len >= mnl) out.push_back(c.v);
        } else {
          kept.push_back(c);
        }
      }
      stack.swap(kept);
      return 0;
    };
    int round = 1;
    if (int need = search(round)) { bynum_need = need; return MINE_RETRY; }
    max_num = std::max(max_num, (int)out.size());
    while ((int)out.size() < max_num && theta > 1e-38) {
      if (stack.empty()) break;  // nothing left to accept: later rounds change nothing
      last_size = (int)out.size();
      theta *= 0.9;
      ++round;
      if (int need = search(round)) { bynum_need = need; return MINE_RETRY; }
    }
    if ((int)out.size() > max_num) {
      std::sort(out.begin() + last_size, out.end(), [&](int32_t x, int32_t y) { return fr[x] > fr[y]; });
      out.resize(max_num);
    }
    std::vector<uint32_t> pos(ntot, 0);
    for (int32_t v = 0; v < ntot; ++v) fl[v] &= (uint8_t)~NODE_ACC;
    for (size_t i = 0; i < out.size(); ++i) {
      fl[out[i]] |= NODE_ACC;
      pos[out[i]] = (uint32_t)i;
    }
    if (ntot > 0 &&
        ((e = hipMemcpyAsync(n_flags.p, fl.data(), (size_t)ntot, hipMemcpyHostToDevice, st)) ||
         (e = hipMemcpyAsync(n_pos.p, pos.data(), (size_t)ntot * 4, hipMemcpyHostToDevice, st)) ||
         (e = hipStreamSynchronize(st))))
      return hipfail(e, "bynum");
    P = (int)out.size();
    rm_out = rm;
    bynum_theta_last = theta;  // m_min_freq after the search (estimatePatterns filters by it)
    return HMC_OK;
  }

  int build_heads_from_nodes(const MineArgs &, int hb, int he) {
    std::vector<std::pair<uint32_t, uint8_t>> heads;
    hf_valid = false;
    h_head_ids.clear();
    h_head_al.clear();
    if (head_len == 1 && pan.L > 0) {
      const int n0 = h_npos[0];
      std::vector<int32_t> rcb(1);
      hipError_t e;
      std::vector<uint8_t> fl(n0), alle(n0);
      std::vector<uint32_t> pos(n0);
      if ((e = hipMemcpyAsync(rcb.data(), d_r_child_base.p, 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipStreamSynchronize(st)))
        return hipfail(e, "heads");
      if (n0 > 0) {
        const long long r0 = (long long)rcb[0] - wbase;  // physical index of root 0's first child
        if ((e = hipMemcpyAsync(fl.data(), n_flags.p + r0, n0, hipMemcpyDeviceToHost, st)) ||
            (e = hipMemcpyAsync(alle.data(), n_allele.p + r0, n0, hipMemcpyDeviceToHost, st)) ||
            (e = hipMemcpyAsync(pos.data(), n_pos.p + r0, (size_t)n0 * 4, hipMemcpyDeviceToHost, st)) ||
            (e = hipStreamSynchronize(st)))
          return hipfail(e, "heads");
      }
      for (int k = 0; k < n0; ++k)
        if (fl[k] & NODE_ACC) heads.push_back({pos[k], alle[k]});
    } else if (head_len > 1 && he > hb) {
      // head list = accepted start-0 nodes of level head_len; their alleles by
      // walking parent links (levels 1..head_len are nodes [0, he))
      hipError_t e;
      std::vector<int32_t> par(he), stt(he);
      std::vector<uint8_t> fl(he), alle(he);
      std::vector<uint32_t> pos(he);
      if ((e = hipMemcpyAsync(par.data(), n_parent.p, (size_t)he * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(stt.data(), n_start.p, (size_t)he * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(fl.data(), n_flags.p, (size_t)he, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(alle.data(), n_allele.p, (size_t)he, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(pos.data(), n_pos.p, (size_t)he * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipStreamSynchronize(st)))
        return hipfail(e, "heads");
      std::vector<std::pair<uint32_t, std::vector<uint8_t>>> hs;
      for (int v = hb; v < he; ++v) {
        if (stt[v] != 0 || !(fl[v] & NODE_ACC)) continue;
        std::vector<uint8_t> al(head_len);
        int32_t w = v;
        for (int q = head_len - 1; q >= 0; --q) {
          al[q] = alle[w];
          w = par[w];
        }
        hs.push_back({pos[v], al});
      }
      std::sort(hs.begin(), hs.end());
      std::vector<uint8_t> tab((size_t)std::max(P, 1) * head_len, 0);
      for (auto &h : hs) {
        heads.push_back({h.first, h.second[head_len - 1]});
        h_head_ids.push_back(h.first);
        h_head_al.insert(h_head_al.end(), h.second.begin(), h.second.end());
        std::copy(h.second.begin(), h.second.end(), tab.begin() + (size_t)h.first * head_len);
      }
      if ((e = d_head_al.ensure(tab.size())) ||
          (e = hipMemcpyAsync(d_head_al.p, tab.data(), tab.size(), hipMemcpyHostToDevice, st)) ||
          (e = hipStreamSynchronize(st)))
        return hipfail(e, "heads");
    }
    return set_heads(heads);
  }

  // initHeadList (HaploBuilder.cpp:153-224) for head_len > 1, on the host: the
  // head pairs of every individual of the shard, in the reference's order
  // (head list in id order; allele sequences expanded locus by locus;
  // findLongestMatchPattern(head_len, as) must give a start-0 pattern).
  int build_head_frontier() {
    const int n = nloc(), hl = head_len;
    const int nh = (int)h_head_ids.size();
    if (nh == 0 && !h_head_al.empty()) return fail(HMC_EARG, "head alleles without heads");
    // the start-0 length-hl pattern matching `as` (MISSING = wildcard): the
    // trie walk of PatternTree.cpp:98-134 goes from locus hl-1 down and keeps
    // the first full-length hit, i.e. the smallest allele index at the
    // highest missing locus first
    auto lookup = [&](const std::vector<uint8_t> &as) -> uint32_t {
      int best = -1;
      for (int h = 0; h < nh; ++h) {
        const uint8_t *al = h_head_al.data() + (size_t)h * hl;
        bool ok = true;
        for (int k = 0; k < hl && ok; ++k) ok = as[k] == MISSING || as[k] == al[k];
        if (!ok) continue;
        if (best < 0) { best = h; continue; }
        const uint8_t *bl = h_head_al.data() + (size_t)best * hl;
        for (int k = hl - 1; k >= 0; --k)
          if (al[k] != bl[k]) {
            if (al[k] < bl[k]) best = h;
            break;
          }
      }
      return best < 0 ? NONE : h_head_ids[best];
    };
    std::vector<uint32_t> off(n + 1, 0), pairs;
    std::vector<int32_t> status(n, EST_OK);
    for (int i = 0; i < n; ++i) {
      off[i] = (uint32_t)(pairs.size() / 2);
      const uint8_t *g0 = pan.idx.data() + ((size_t)(i0 + i) * 2) * pan.L, *g1 = g0 + pan.L;
      for (int h = 0; h < nh && status[i] == EST_OK; ++h) {
        const uint8_t *H = h_head_al.data() + (size_t)h * hl;
        bool match = true;  // HaploPattern::isMatch(genotype): every locus matches one allele
        for (int j = 0; j < hl && match; ++j)
          match = g0[j] == MISSING || g1[j] == MISSING || g0[j] == H[j] || g1[j] == H[j];
        if (!match) continue;
        std::vector<std::vector<uint8_t>> last(1), next;
        for (int j = 0; j < hl; ++j) {
          next.clear();
          const bool miss0 = g0[j] == MISSING, miss1 = g1[j] == MISSING;
          const bool isMissing = miss0 && miss1, hasMissing = miss0 || miss1;
          const bool hasAllele = g0[j] == H[j] || g1[j] == H[j];  // Allele == (missing == missing)
          const bool het = !(hasMissing || g0[j] == g1[j]);
          if (isMissing || (hasMissing && hasAllele)) {
            for (auto &as : last)
              for (int k = 0; k < (int)pan.sym[j].size(); ++k)
                if (pan.sym[j][k].second > 0) {
                  next.push_back(as);
                  next.back().push_back((uint8_t)k);
                }
          } else if (het) {
            for (auto &as : last) {
              next.push_back(as);
              next.back().push_back(H[j] == g0[j] ? g1[j] : g0[j]);
            }
          } else {
            for (auto &as : last) {
              next.push_back(as);
              next.back().push_back(g0[j]);
            }
          }
          last.swap(next);
        }
        for (auto &as : last) {
          const uint32_t q = lookup(as);
          if (q == NONE) { status[i] = EST_NO_HEAD_PATTERN; break; }
          if (q >= h_head_ids[h]) {
            pairs.push_back(h_head_ids[h]);
            pairs.push_back(q);
          }
        }
      }
    }
    off[n] = (uint32_t)(pairs.size() / 2);
    hipError_t e;
    if ((e = d_hf_off.ensure(n + 1)) || (e = d_hf_pairs.ensure(std::max<size_t>(pairs.size(), 2))) ||
        (e = d_hf_status.ensure(std::max(n, 1))) ||
        (e = hipMemcpyAsync(d_hf_off.p, off.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice, st)) ||
        (!pairs.empty() && (e = hipMemcpyAsync(d_hf_pairs.p, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice, st))) ||
        (n && (e = hipMemcpyAsync(d_hf_status.p, status.data(), (size_t)n * 4, hipMemcpyHostToDevice, st))) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "head frontier");
    hf_valid = true;
    return HMC_OK;
  }

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
  int estep(double *ll_out, int *H_out, uint64_t *re_out) {
    if (!have_model) return fail(HMC_EARG, "no pattern model");
    if (head_len > 1) {
      if (h_head_al.size() != h_head_ids.size() * (size_t)head_len || (h_head_ids.empty() && n_head > 0))
        return fail(HMC_EUNSUPPORTED, "head_len > 1 needs the head patterns' alleles (mined tables only)");
      int rc = build_head_frontier();
      if (rc) return rc;
    }
    const int L = pan.L, S = this->S(), n = nloc();
    if (S > S_MAX) return fail(HMC_EUNSUPPORTED, "sample_size > %d", S_MAX);
    if (S > 32 && estep_mode != ESTEP_SPLIT)
      return fail(HMC_EUNSUPPORTED, "sample_size > 32 needs the split E-step (hmc_set_estep_mode 0)");
    hipError_t e;
    if ((e = d_total.ensure(n)) || (e = d_ncand.ensure(n)) || (e = d_status.ensure(n)) || (e = d_re.ensure(n)) ||
        (e = d_sbase.ensure(n)) || (e = d_prior.ensure((size_t)n * S_MAX)) || (e = d_post.ensure((size_t)n * S_MAX)) ||
        (e = d_weight.ensure((size_t)n * S_MAX)) || (e = d_cstate.ensure((size_t)n * S_MAX)) ||
        (e = d_cidx.ensure((size_t)n * S_MAX)) || (e = d_rows.ensure((size_t)2 * S * n * L)) ||
        (e = d_wslot.ensure((size_t)2 * S * n)) || (e = d_trace_cursor.ensure(1)) || (e = d_maxst.ensure(1)) ||
        (e = d_fmax.ensure(n)) || (e = d_loc_off.ensure((size_t)n * (L + 1))) || (e = d_order.ensure(n)) ||
        (e = d_order2.ensure(n)) || (e = d_cost.ensure(n)) || (e = d_tbase.ensure(n)) || (e = d_rbase.ensure(n)) ||
        (e = d_rneed.ensure(n)) || (e = d_tneed.ensure(n)) || (e = d_recsz.ensure(n)))
      return hipfail(e, "estep alloc");
    // store budgets: trace store and record store grow (never shrink) up to these
    size_t freeb = 0, totb = 0;
    hipMemGetInfo(&freeb, &totb);
    const double avail = (double)freeb + (double)d_trace.n * 4 + (double)d_rec.n * 4;
    // Frontier capacity of the structure pass: a frontier past it restarts the
    // E-step with twice the capacity (cfg 3's E1 on the M0 model needs 2^14:
    // three restarts from 2^11, ~0.6 s).  With HBM to spare, start there: the
    // pass's per-block scratch is ~190 B per state (3 GB per 1 000 blocks).
    if (!fcap_user_set && fcap < FCAP_BIG && avail > 96e9) fcap = FCAP_BIG;
    // (cfg 3's E1 with the M0 model needs ~2x HBM in records + traces; larger
    // stores (fewer groups) measured no faster and crowd out the next M0.  The
    // trace cap keeps cfg 3's E2.. (~90 GB of traces) in one value pass.)
    trace_budget = std::max<uint64_t>(trace_bytes ? trace_bytes : std::min<uint64_t>((uint64_t)(avail * 0.42), 120ull << 30),
                                      1ull << 16) / 4;
    rec_budget = std::max<uint64_t>(rec_bytes ? rec_bytes : trace_bytes ? trace_bytes
                                    : std::min<uint64_t>((uint64_t)(avail * 0.28), 80ull << 30),
                                    1ull << 16) / 4;
    if (debug_mem)
      fprintf(stderr, "[hmc] E-step: free %.1f GB, stores %.1f + %.1f GB, budgets trace %.1f rec %.1f GB\n",
              freeb / 1e9, d_trace.n * 4 / 1e9, d_rec.n * 4 / 1e9, trace_budget * 4 / 1e9, rec_budget * 4 / 1e9);
    // Stores sized by an earlier E-step when more HBM was free (E1, before an
    // exact M-step's tables) shrink to this E-step's budgets: the pass
    // scratch is allocated from what they leave free.
    if (d_trace.n > trace_budget) d_trace.release();
    if (d_rec.n > rec_budget) d_rec.release();
    h_total.assign(n, 0.0);
    h_ncand.assign(n, 0);
    h_status.assign(n, 0);
    h_re.assign(n, 0);
    h_sbase.assign(n, 0);
    for (int i = 0; i < n; ++i) h_sbase[i] = 2 * S * i;  // sample slots of individual i
    if ((e = hipMemcpyAsync(d_sbase.p, h_sbase.data(), (size_t)n * 4, hipMemcpyHostToDevice, st)) ||
        (e = hipMemsetAsync(d_maxst.p, 0, 4, st)) || (e = hipMemsetAsync(d_ncand.p, 0, (size_t)n * 4, st)))
      return hipfail(e, "estep");
    if ((e = d_stamps.ensure(40)) || (e = hipMemsetAsync(d_stamps.p, 0, 40 * 8, st))) return hipfail(e, "stamps");
    // heaviest individuals first (cost of the previous E-step; before the
    // first one, the number of heterozygous or missing loci)
    if ((int)h_cost.size() != n) {
      h_cost.assign(n, 0);
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < L; ++k) {
          const uint8_t x = pan.idx[((size_t)(i0 + i) * 2) * L + k], y = pan.idx[((size_t)(i0 + i) * 2 + 1) * L + k];
          h_cost[i] += (x != y || x == MISSING) ? 1 : 0;
        }
    }
    std::vector<int32_t> order(n);
    for (int q = 0; q < n; ++q) order[q] = q;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return h_cost[x] > h_cost[y]; });
    if ((e = hipMemcpyAsync(d_cost.p, h_cost.data(), (size_t)n * 4, hipMemcpyHostToDevice, st)))
      return hipfail(e, "estep");
    ms_fwd = ms_tb = 0;
    ms_s1 = ms_s2 = ms_fb = ms_order = 0;
    n_fallback = n_order_redo = 0;
    n_struct_passes = n_value_passes = 0;
    int rc = 0;
    while (true) {  // a frontier overflow (fcap grows) restarts the E-step
      rc = estep_mode == ESTEP_SPLIT ? estep_split(order) : estep_fused(order);
      if (rc != ESTEP_RESTART) break;
    }
    if (rc) return rc;
    if (estep_mode == ESTEP_SPLIT) ms_fwd = ms_s1 + ms_s2 + ms_fb;
    // samples in the reference's order: individuals in order, candidates in
    // order, h0 then h1 (HaploModel.cpp:105-106)
    std::vector<int32_t> rowmap;
    rowmap.reserve((size_t)2 * S * n);
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < 2 * h_ncand[i]; ++c) rowmap.push_back(h_sbase[i] + c);
    H = (int)rowmap.size();
    std::vector<double> wslot((size_t)2 * S * n), w(H);
    if ((e = d_samp_lm.ensure((size_t)std::max(H, 1) * L)) || (e = d_rowmap.ensure(std::max(H, 1))) ||
        (e = d_w.ensure(std::max(H, 1))))
      return hipfail(e, "samples");
    if ((H && (e = hipMemcpyAsync(d_rowmap.p, rowmap.data(), (size_t)H * 4, hipMemcpyHostToDevice, st))) ||
        (e = launch_transpose_rows_u8(d_rows.p, d_rowmap.p, d_samp_lm.p, H, L, st)) ||
        (e = hipMemcpyAsync(wslot.data(), d_wslot.p, wslot.size() * 8, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(h_total.data(), d_total.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(h_re.data(), d_re.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
        (e = hipMemcpyAsync(h_cost.data(), d_cost.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "estep");
    for (int h = 0; h < H; ++h) w[h] = wslot[rowmap[h]];
    if (H && ((e = hipMemcpyAsync(d_w.p, w.data(), (size_t)H * 8, hipMemcpyHostToDevice, st)) ||
              (e = hipStreamSynchronize(st))))
      return hipfail(e, "estep");
    h_rowmap.swap(rowmap);
    // ll += log(genotype probability) in individual order (HaploModel.cpp:110);
    // HaploData::checkTotalWeight (HaploData.cpp:120-126) in sample order
    double red[2] = {0.0, 0.0};
    auto local_sums = [&](double *acc) {
      double ll = acc[0], tw = acc[1];
      for (int i = 0; i < n; ++i) ll += log(h_total[i]);
      for (int h = 0; h < H; ++h) tw += w[h];
      acc[0] = ll;
      acc[1] = tw;
    };
    if (multi() && reduction == RED_ORDERED) {
      for (int r = 0; r < world; ++r) {  // the chain continues rank by rank
        if (r == rank) local_sums(red);
        if ((rc = bcast_host(red, 2, r))) return rc;
      }
    } else {
      local_sums(red);
      if ((rc = allreduce_host(red, 2))) return rc;
    }
    const double ll = red[0];
    total_weight = red[1];
    uint64_t re = 0;
    for (int i = 0; i < n; ++i) re += h_re[i];
    have_samples = true;
    have_estep = true;
    if (ll_out) *ll_out = ll;
    if (H_out) *H_out = H;
    if (re_out) *re_out = re;
    return HMC_OK;
  }

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
  int ensure_store(DevBuf<uint32_t> &b, uint64_t words, uint64_t budget, const char *what) {
    if (b.n >= words && b.p) return HMC_OK;
    if (words > budget) return fail(HMC_ENOMEM, "%s: one individual needs %llu words (budget %llu)", what,
                                    (unsigned long long)words, (unsigned long long)budget);
    b.release();  // 1.25x headroom: a store of tens of GB is mapped eagerly, re-allocations are slow
    const uint64_t want = std::min<uint64_t>(budget, words + words / 4);
    hipError_t e = b.ensure(want);
    if (e == hipErrorOutOfMemory && want > words) {  // the device is shared: no headroom
      (void)hipGetLastError();
      e = b.ensure(words);
    }
    if (e) return hipfail(e, what);
    return HMC_OK;
  }

  EstepArgs estep_args(int S) {
    EstepArgs a;
    a.pan = dev_panel();
    a.mod = dev_model();
    a.S = S;
    a.indiv_begin = i0;
    a.indiv_end = i1;
    a.scratch = d_scratch.p;
    a.fcap = fcap;
    a.hcap = next_pow2(2 * fcap);
    a.scratch_stride = estep_scratch_bytes(fcap, a.hcap, S, estep_nw);
    lds_tier(S, a.lds_fc, a.lds_hc);
    a.trace = d_trace.p;
    a.trace_cap = d_trace.n;
    a.trace_cursor = d_trace_cursor.p;
    a.trace_base = nullptr;
    a.loc_off = d_loc_off.p;
    a.total = d_total.p;
    a.ncand = d_ncand.p;
    a.status = d_status.p;
    a.cand_state = d_cstate.p;
    a.cand_idx = d_cidx.p;
    a.prior = d_prior.p;
    a.posterior = d_post.p;
    a.weight = d_weight.p;
    a.re_count = d_re.p;
    a.max_states = d_maxst.p;
    a.fmax = d_fmax.p;
    a.order = nullptr;
    a.n_order = 0;
    a.cost = d_cost.p;
    a.stamps = d_stamps.p;
    a.diag_indiv = -1;  // diagnostic build: stamps of every individual
    return a;
  }

  int upload_order(DevBuf<int32_t> &d, const int32_t *v, int k) {
    hipError_t e;
    if (k > 0 && ((e = hipMemcpyAsync(d.p, v, (size_t)k * 4, hipMemcpyHostToDevice, st)) ||
                  (e = hipStreamSynchronize(st))))
      return hipfail(e, "estep order");
    return HMC_OK;
  }

  // Traceback of the individuals in d_order2[0, k) into their sample slots.
  int traceback_group(int k) {
    TracebackArgs t;
    t.L = pan.L;
    t.S = S();
    t.head_len = head_len;
    t.nbatch = k;
    t.order = d_order2.p;
    t.indiv_begin = i0;
    t.mod = dev_model();
    t.trace = d_trace.p;
    t.loc_off = d_loc_off.p;
    t.ncand = d_ncand.p;
    t.cand_state = d_cstate.p;
    t.cand_idx = d_cidx.p;
    t.weight = d_weight.p;
    t.sample_base = d_sbase.p;
    t.rows = d_rows.p;
    t.w_out = d_wslot.p;
    hipError_t e;
    hipEventRecord(ev[2], st);
    if ((e = launch_traceback(t, 0, st))) return hipfail(e, "traceback");
    hipEventRecord(ev[3], st);
    if ((e = hipStreamSynchronize(st))) return hipfail(e, "traceback");
    float ms = 0;
    hipEventElapsedTime(&ms, ev[2], ev[3]);
    ms_tb += ms;
    return HMC_OK;
  }

  int read_status(const std::vector<int32_t> &ids, int k, bool ncand, const int32_t *dstatus = nullptr) {
    // per-individual status (and candidate counts) of ids[0, k): whole arrays, small
    hipError_t e;
    const int n = nloc();
    if ((e = hipMemcpyAsync(h_status.data(), dstatus ? dstatus : d_status.p, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        (ncand && (e = hipMemcpyAsync(h_ncand.data(), d_ncand.p, (size_t)n * 4, hipMemcpyDeviceToHost, st))) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "estep status");
    (void)ids;
    (void)k;
    return HMC_OK;
  }

  // Fused single-pass E-step (estep.hip) over `pending`: trace sizes are not
  // known in advance, so groups are tried and halved on a trace overflow.
  int estep_fused(const std::vector<int32_t> &order) {
    const int S = this->S(), n = nloc();
    int dev_cu = 256;
    hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
    const int G = std::max(1, std::min(waves > 0 ? waves : dev_cu * std::max(8, lds_waves_per_cu), n));
    hipError_t e;
    size_t pos = 0;
    int batch = n;
    if (d_trace.n == 0) {
      int rc = ensure_store(d_trace, std::min<uint64_t>(trace_budget, std::max<uint64_t>((uint64_t)n * pan.L * (1 + S) * 96, 16ull << 20)),
                            trace_budget, "trace store");
      if (rc) return rc;
    }
    while (pos < order.size()) {
      const int k = (int)std::min<size_t>(batch, order.size() - pos);
      EstepArgs a = estep_args(S);
      const int grid = std::min(G, k);
      if ((e = d_scratch.ensure(a.scratch_stride * grid))) return hipfail(e, "estep scratch");
      a.scratch = d_scratch.p;
      int rc = upload_order(d_order2, order.data() + pos, k);
      if (rc) return rc;
      a.order = d_order2.p;
      a.n_order = k;
      if ((e = hipMemsetAsync(d_trace_cursor.p, 0, 8, st))) return hipfail(e, "estep");
      hipEventRecord(ev[0], st);
      if ((e = launch_estep(a, grid, estep_nw, st))) return hipfail(e, "estep_forward launch");
      hipEventRecord(ev[1], st);
      if ((rc = read_status(order, k, true))) return rc;
      float ms = 0;
      hipEventElapsedTime(&ms, ev[0], ev[1]);
      ms_fwd += ms;
      bool ovf_trace = false;
      for (int q = 0; q < k; ++q) {
        const int s = h_status[order[pos + q]];
        if (s == EST_NO_HEAD_PATTERN) return fail(HMC_ENOPATTERN, "Can not find matching pattern!");
        if (s == EST_OVERFLOW_FRONTIER) {
          if (fcap >= F_MAX) return fail(HMC_EUNSUPPORTED, "frontier exceeds %d states", F_MAX);
          fcap = (int)std::min<int64_t>(F_MAX, (int64_t)fcap * 4);  // x4: each overflow costs a whole pass
          return ESTEP_RESTART;
        }
        if (s == EST_OVERFLOW_TRACE) ovf_trace = true;
      }
      if (ovf_trace) {
        if (d_trace.n < trace_budget) {  // grow the store before splitting the group
          if ((rc = ensure_store(d_trace, std::min<uint64_t>(trace_budget, d_trace.n * 4), trace_budget, "trace store")))
            return rc;
          continue;
        }
        if (k == 1) return fail(HMC_ENOMEM, "trace store too small for one individual");
        batch = std::max(1, k / 2);
        continue;
      }
      if ((rc = traceback_group(k))) return rc;
      pos += k;
    }
    return HMC_OK;
  }

  // Split E-step (estep_split.hip): structure pass, value pass, fused fallback
  // for individuals whose forward likelihood underflows.
  // exact = true: the exact M-step's pass over the individuals (structure
  // records with forward links, then exact_fb + exact_walk per group instead
  // of the value pass and traceback; E-step outputs are left untouched).
  int estep_split(const std::vector<int32_t> &order, bool exact = false) {
    const int S = this->S(), n = nloc(), L = pan.L;
    int32_t *dstatus = exact ? d_xstatus.p : d_status.p;
    int dev_cu = 256;
    hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, device);
    const int G = std::max(1, std::min(waves > 0 ? waves : dev_cu * std::max(8, lds_waves_per_cu), n));
    hipError_t e;
    float ms = 0;
    std::vector<int32_t> pending(order), sset, rest;
    std::vector<unsigned long long> rneed(n, 0), tneed(n, 0), base(n, 0), rsz(n, 0);
    std::vector<int32_t> fbig(n, 0);  // largest frontier of each individual (structure pass)
    // Every individual gets its own record region: its exact size once a pass
    // has measured it (`exact_need`), else an estimate — the previous E-step's
    // size when the model is of the same scale, or the records-per-cost ratio
    // of the individuals measured so far.  A region that turns out too small
    // only defers that individual (it keeps walking without writing and
    // reports its exact size), so no pass is ever repeated in full.
    std::vector<char> exact_need(n, 0);
    std::vector<unsigned long long> est(n, 0);
    const bool prev_ok = !exact && (int)prev_rneed.size() == n && prev_P > 0 && P < 2 * (int64_t)prev_P &&
                         2 * (int64_t)P > prev_P;
    if (prev_ok)
      for (int i = 0; i < n; ++i) est[i] = prev_rneed[i] + prev_rneed[i] / 10 + 64;
    bool have_est = prev_ok;
    int rc;
    while (!pending.empty()) {
      // ---- pass 1: structure records --------------------------------------
      int np = (int)pending.size();
      {
        uint64_t r = 0, t = 0;
        int k = 0;
        // the first pass spans the whole cost range and later estimates use the
        // measured individuals nearest in cost (cfg 3 E1 after E5: 7.1 -> 5.9 s,
        // deferred 1 713 -> 12 per group, profiles/r02/e1_groups/)
        if (!have_est) {  // nothing measured yet: 4 per CU share the store evenly
          k = std::min(np, 4 * dev_cu);
          if (np > k) {  // every np/k-th of the heaviest-first list
            std::vector<int32_t> pick, other;
            pick.reserve(k);
            other.reserve(np - k);
            for (int q = 0; q < np; ++q)
              ((int64_t)q * k / np != (int64_t)(q - 1) * k / np || q == 0 ? pick : other).push_back(pending[q]);
            pending = pick;
            pending.insert(pending.end(), other.begin(), other.end());
            k = (int)pick.size();
          }
          const uint64_t share = rec_budget / (uint64_t)k;
          for (int q = 0; q < k; ++q) {
            base[pending[q]] = (uint64_t)q * share;
            rsz[pending[q]] = share;
          }
          r = share * (uint64_t)k;
        } else {  // the prefix whose regions (and measured traces) fit the budgets
          uint64_t r_est = 0;
          while (k < np) {
            const int bi = pending[k];
            const uint64_t need = exact_need[bi] ? rneed[bi] : std::min<uint64_t>(est[bi], rec_budget);
            // (estimated traces are not counted: groups cut by records and then
            // split by exact traces measured faster at cfg 3's E1)
            const uint64_t tn = exact_need[bi] ? tneed[bi] : 0;
            if (k > 0 && (r + need > rec_budget || t + tn > trace_budget)) break;
            rsz[bi] = need;
            r += need;
            t += tn;
            r_est += exact_need[bi] ? 0 : need;
            ++k;
          }
          // the store left over goes to the estimated regions (up to 3x), so
          // fewer individuals are deferred to a pass of their own (A/B on one
          // box, cfg 3: E1 value passes 3.88 -> 3.60 s, E2 structure 218 -> 177 ms)
          const double grow = r_est > 0 && r < rec_budget
                                  ? std::min(3.0, 1.0 + (double)(rec_budget - r) / (double)r_est)
                                  : 1.0;
          r = 0;
          for (int q = 0; q < k; ++q) {
            const int bi = pending[q];
            if (!exact_need[bi]) rsz[bi] = std::min<uint64_t>((uint64_t)((double)rsz[bi] * grow), rec_budget);
            if (r + rsz[bi] > rec_budget) rsz[bi] = rec_budget - r;
            base[bi] = r;
            r += rsz[bi];
          }
        }
        np = k;
        rec_words = r;
        std::vector<unsigned long long> rb(n, 0), rs(n, 0);
        for (int q = 0; q < np; ++q) {
          rb[pending[q]] = base[pending[q]];
          rs[pending[q]] = rsz[pending[q]];
        }
        if ((e = hipMemcpyAsync(d_rbase.p, rb.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) ||
            (e = hipMemcpyAsync(d_recsz.p, rs.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)))
          return hipfail(e, "estep");
      }
      const int hcap1 = next_pow2(2 * fcap);
      // (exact records pack a locus's contribution count in 22 bits, R[3] = C << 10 | npairs)
      const int ccap1 = (int)std::min<int64_t>(exact ? EXACT_C_MAX : INT32_MAX / 2, (int64_t)ccap_mult * fcap);
      // Structure pass over ids[0, np_) in the record regions set above (d_rbase /
      // d_recsz).  prune_: with extend()'s forward test (HaploBuilder.cpp:237),
      // for the individuals the value pass found underflowing.
      auto structure_pass = [&](const int32_t *ids, int np_, bool prune_) -> int {
        int rc;
        hipError_t e;
        float ms = 0;
        // structure pass: one wave per individual; 12 per CU (3 per SIMD at 145
        // VGPRs) above 8 per CU, so cfg 3's E1 groups of 2 200-2 700 run in one
        // round (profiles/r02/e1_groups/: 603-658 -> 484-586 ms per group).  On a
        // model larger than the panel (the genotype-mined M0: 2.5 patterns per
        // individual-locus at cfg 3, 0.3 later) frontiers are large (cfg 3 E1:
        // 470 states per locus, 80 % of them past a one-wave block's LDS tier):
        // four waves per individual, two per CU (each block's LDS tier holds
        // more of the frontier: cfg 3 E1 structure 1.65 -> 1.32 s against three
        // per CU, profiles/r03/e1/e1_s1shapes.log)
        const bool heavy_model = (double)P > (double)pan.N * (double)pan.L;
        // (a heavy group of at most one individual per CU — cfg 4's per-rank E1,
        // records of ~250 MB per individual — takes the whole CU: 16 waves)
        const int nw1 = s1_nw > 0 ? s1_nw : (heavy_model ? (np_ <= dev_cu ? 16 : 4) : 1);
        const int bpc1 = s1_ipc > 0 ? s1_ipc
                                    : (nw1 == 16 ? 1 : (nw1 == 4 ? 2 : (np_ > 8 * dev_cu ? 12 : (np_ > 4 * dev_cu ? 8 : 4))));
        const size_t per1 = estep_s1_scratch_bytes(fcap, hcap1, ccap1, nw1, prune_);
        // (huge frontiers: fewer resident individuals rather than scratch past SCRATCH_MAX)
        const int grid1 = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::min(np_, dev_cu * bpc1), SCRATCH_MAX / per1));
        // the scratch first: both stores are dead here (the groups before have
        // been traced back), so they give way to it when HBM is short
        // (a prune re-run runs between a value pass and its traceback: both stores are live)
        if ((e = scratch_ensure(d_scr1, per1 * grid1, !prune_, !prune_)) || (e = d_rec_off.ensure((size_t)n * (L + 1))) ||
            (e = d_rec_cursor.ensure(1)) || (e = hipMemsetAsync(d_rec_cursor.p, 0, 8, st)))
          return hipfail(e, "estep pass-1 alloc");
        if ((rc = ensure_store(d_rec, rec_words, rec_budget, "record store"))) return rc;
        if ((rc = upload_order(d_order, ids, np_))) return rc;
        StructArgs s1;
        s1.pan = dev_panel();
        s1.mod = dev_model();
        s1.S = S;
        s1.indiv_begin = i0;
        s1.order = d_order.p;
        s1.n_order = np_;
        s1.scratch = d_scr1.p;
        s1.scratch_stride = per1;
        s1.fcap = fcap;
        s1.hcap = hcap1;
        s1.ccap = ccap1;
        s1_tier(160 * 1024 / bpc1 - 256, pan.amax, nw1, s1.lds_fc, s1.lds_hc, s1.lds_cc);
        s1.rec = d_rec.p;
        s1.rec_cap = d_rec.n;
        s1.rec_cursor = d_rec_cursor.p;
        s1.rec_base = d_rbase.p;
        s1.rec_size = d_recsz.p;
        s1.rec_off = d_rec_off.p;
        s1.rec_need = d_rneed.p;
        s1.trace_need = d_tneed.p;
        s1.status = dstatus;
        s1.re_count = exact ? d_xre.p : d_re.p;
        s1.fmax = exact ? d_xfmax.p : d_fmax.p;
        s1.max_states = d_maxst.p;
        s1.stamps = d_stamps.p + 20;
        s1.exact = exact;
        s1.prune = prune_;
        if ((e = d_nextq.ensure(2)) || (e = hipMemsetAsync(d_nextq.p, 0, 8, st))) return hipfail(e, "estep");
        s1.next_q = d_nextq.p;
        hipEventRecord(ev[0], st);
        if ((e = launch_estep_structure(s1, grid1, nw1, st))) return hipfail(e, "estep_structure launch");
        hipEventRecord(ev[1], st);
        if ((e = hipMemcpyAsync(rneed.data(), d_rneed.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
            (e = hipMemcpyAsync(tneed.data(), d_tneed.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) ||
            (e = hipMemcpyAsync(fbig.data(), s1.fmax, (size_t)n * 4, hipMemcpyDeviceToHost, st)))
          return hipfail(e, "estep_structure");
        if ((rc = read_status(pending, np_, false, dstatus))) return rc;
        hipEventElapsedTime(&ms, ev[0], ev[1]);
        if (prune_) {
          ms_fb += ms;
        } else {
          ms_s1 += ms;
          ++n_struct_passes;
        }
        return HMC_OK;
      };
      if ((rc = structure_pass(pending.data(), np, false))) return rc;
      if (debug_mem) {
        int ndef = 0;
        uint64_t rsum = 0, rmax = 0, tsum = 0, rres = 0;
        for (int q = 0; q < np; ++q) {
          const int bi = pending[q];
          ndef += h_status[bi] == EST_OVERFLOW_REC ? 1 : 0;
          rsum += rneed[bi];
          rmax = std::max<uint64_t>(rmax, rneed[bi]);
          tsum += tneed[bi];
          rres += rsz[bi];
        }
        fprintf(stderr, "[hmc] structure pass %d: %d individuals, %.1f ms; deferred %d, records need %.2f GB (max %.1f MB, "
                "reserved %.2f GB), traces %.2f GB\n", n_struct_passes, np, ms, ndef, rsum * 4e-9, rmax * 4e-6, rres * 4e-9,
                tsum * 4e-9);
      }
      sset.clear();
      rest.clear();
      for (int q = 0; q < np; ++q) {
        const int bi = pending[q], s = h_status[bi];
        if (s == EST_NO_HEAD_PATTERN) return fail(HMC_ENOPATTERN, "Can not find matching pattern!");
        if (s == EST_OVERFLOW_CONTRIB) {  // missing genotypes: up to amax^2 contributions per state
          if ((int64_t)ccap_mult * fcap >= INT32_MAX / 2) return fail(HMC_EUNSUPPORTED, "too many contributions at a locus");
          if (exact && ccap1 >= EXACT_C_MAX)
            return fail(HMC_EUNSUPPORTED, "exact M-step: more than %d contributions at a locus", EXACT_C_MAX);
          ccap_mult *= 2;
          return ESTEP_RESTART;
        }
        if (s == EST_OVERFLOW_FRONTIER) {  // (deferring only these individuals measured slower)
          if (fcap >= F_MAX) return fail(HMC_EUNSUPPORTED, "frontier exceeds %d states", F_MAX);
          if (debug_mem) fprintf(stderr, "[hmc] frontier over %d states: capacity x4, E-step restarts\n", fcap);
          fcap = (int)std::min<int64_t>(F_MAX, (int64_t)fcap * 4);  // x4: each overflow costs a whole pass
          return ESTEP_RESTART;
        }
        if (s == EST_OVERFLOW_REC) {
          if (exact_need[bi]) return fail(HMC_EHIP, "record store overflow with exact sizes");
          rest.push_back(bi);
        } else {
          sset.push_back(bi);
        }
        exact_need[bi] = 1;
      }
      for (int q = np; q < (int)pending.size(); ++q) rest.push_back(pending[q]);
      // estimates for the individuals not measured yet: records per unit of
      // cost of those measured (after a pass where estimates fell short, or
      // when there were none)
      {
        int deferred = 0;
        double rs_ = 0, cs = 0;
        for (int i = 0; i < n; ++i)
          if (exact_need[i]) {
            rs_ += (double)rneed[i];
            cs += (double)std::max(1, h_cost[i]);
          }
        for (int q = 0; q < np; ++q) deferred += h_status[pending[q]] == EST_OVERFLOW_REC ? 1 : 0;
        if (!have_est || deferred * 10 > np) {
          const double ratio = cs > 0 ? rs_ / cs : 0.0;
          std::vector<std::pair<int, double>> cr;  // (cost, records per cost) of the measured
          for (int i = 0; i < n; ++i)
            if (exact_need[i]) cr.emplace_back(std::max(1, h_cost[i]), (double)rneed[i] / std::max(1, h_cost[i]));
          std::sort(cr.begin(), cr.end());
          for (int bi : rest) {
            if (exact_need[bi]) continue;
            const int c = std::max(1, h_cost[bi]);
            if (cr.empty()) {
              est[bi] = (uint64_t)(1.25 * ratio * c) + 64;
              continue;
            }
            // the largest ratio among the 4 measured nearest in cost on each side
            const int at = (int)(std::lower_bound(cr.begin(), cr.end(), std::make_pair(c, -1.0)) - cr.begin());
            double q = 0.0;
            for (int u = std::max(0, at - 4); u < std::min((int)cr.size(), at + 4); ++u) q = std::max(q, cr[u].second);
            est[bi] = (uint64_t)(1.1 * q * c) + 64;
          }
          have_est = true;
        }
      }
      // ---- pass 2: values, in groups whose traces fit the store -------------
      size_t pos = 0;
      while (pos < sset.size()) {
        uint64_t t = 0;
        size_t k = 0;
        while (pos + k < sset.size() && (k == 0 || t + tneed[sset[pos + k]] <= trace_budget)) {
          base[sset[pos + k]] = t;
          t += tneed[sset[pos + k]];
          ++k;
        }
        // traces over the budget by a few individuals while structure groups
        // still follow: those join the next group (re-walked there, exact sizes
        // known) instead of a value pass of their own, which would cost one
        // heavy individual's whole latency (cfg 3 E1: 61-78 individuals,
        // 230-270 ms each, profiles/r02/e1_groups/)
        if (pos == 0 && !exact && !rest.empty() && k < sset.size() && 4 * (sset.size() - k) <= sset.size()) {
          rest.insert(rest.begin(), sset.begin() + (std::ptrdiff_t)k, sset.end());
          sset.resize(k);
        }
        if ((rc = ensure_store(d_trace, std::max<uint64_t>(t, 1), trace_budget, "trace store"))) return rc;
        std::vector<unsigned long long> tb(n, 0);
        for (size_t q = 0; q < k; ++q) tb[sset[pos + q]] = base[sset[pos + q]];
        if ((e = hipMemcpyAsync(d_tbase.p, tb.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)))
          return hipfail(e, "estep");
        if ((rc = upload_order(d_order2, sset.data() + pos, (int)k))) return rc;
        if (exact) {
          // individuals whose forward likelihood underflows: records rebuilt with
          // extend()'s forward test (HaploBuilder.cpp:237, 291-314) before the walk
          auto rerun = [&](std::vector<int32_t> &ids) { return structure_pass(ids.data(), (int)ids.size(), true); };
          if ((rc = exact_group(sset.data() + pos, (int)k, rerun))) return rc;
          pos += k;
          continue;
        }
        // by individuals per CU (cfg 3 and its rank shards, tools/shard_shapes.py,
        // profiles/r02/shard_shapes/): 1:16 from 32 per CU (10 000: 557 vs 615 ms
        // at 2:8), 2:8 from 8 (4 994: 290 vs 333 ms at 1:16), else 3:8 (1 239:
        // 101 vs 112 ms at 2:8)
        // (1:20 runs the 5-waves-per-SIMD build: 505-514 vs 535-558 ms at
        // 1:16 for cfg 3's E3, profiles/r02/values_ab/)
        // Heavy individuals (the first E-step on the genotype-mined model: cfg 3's
        // E1 averages ~3 000 record words per locus against ~650 later) take 4
        // waves each, 4 per CU: more selection segments per individual and a
        // 4x larger LDS frontier tier (cfg 3 E1 value passes 3.84 -> 2.99 s,
        // profiles/r03/e1_shapes/).
        double rw = 0;
        for (size_t q = 0; q < k; ++q) rw += (double)rneed[sset[pos + q]];
        const bool heavy = rw / ((double)k * L) > 1500.0;
        // Heavy groups too small to give every CU four individuals (records and
        // traces of hundreds of MB each: cfg 4's per-rank E1 on the 720 M-pattern
        // M0 runs in groups of ~200) spread the CU's 16 waves over fewer
        // individuals: more selection segments and LDS per individual.
        const int per_cu = (int)((k + dev_cu - 1) / dev_cu);
        const bool small_heavy = heavy && per_cu < 4;
        // (heavy groups filling the GPU: 8 waves x 2 per CU, cfg 3 E1 values
        // 2.95 -> 2.68 s against 4 x 4, profiles/r03/e1/e1_wide.log)
        int vnw = vp_nw > 0 ? vp_nw
                            : (small_heavy ? 16 / per_cu
                                           : (heavy ? 8 : ((int)k >= 32 * dev_cu ? 1 : ((int)k >= 8 * dev_cu ? 2 : 3))));
        int vipc = vp_ipc > 0 ? vp_ipc
                              : (small_heavy ? per_cu
                                             : (vnw == 1 ? 20 : (vnw >= 8 ? 2 : (vnw >= 4 ? 4 : 8))));  // a half-given shape completes by the same rule
        // the HBM tier of the value frontiers holds the group's largest
        // frontier (pass 1 measured it), not the structure pass's capacity
        int fgrp = 1;
        for (size_t q = 0; q < k; ++q) fgrp = std::max(fgrp, (int)fbig[sset[pos + q]]);
        fgrp = std::min(fcap, (fgrp + 63) & ~63);
        // two links per lane (cfg 3: E1 values 2.68 -> 2.34 s, E2 ~3 % less)
        const bool pair = !value_fast && S <= 16 && (value_pair == 2 || (value_pair == 1 && heavy));
        // Dataflow value pass (estep_df.hip): one wave walks the loci and
        // builds the lists, the others run the chains of adds of any open locus.
        DfShape df;
        const bool use_df = !value_fast && S <= 32 && (value_pass == VP_DATAFLOW || (value_pass == VP_AUTO && df_auto(heavy))) &&
                            df_shape(S, pair, heavy, small_heavy, per_cu, fgrp, df);
        if (use_df) {
          vnw = df.nw;
          vipc = df.ipc;
        }
        const int G2 = std::max(1, std::min(waves > 0 ? waves : dev_cu * vipc, n));
        // register budget: 5 waves per SIMD once the shape asks for more than 16 per CU
        const int vwpe = vnw * vipc > 16 && vnw * vipc <= 20 ? 5 : 4;
        const size_t per2 = use_df ? estep_df_scratch_bytes(fgrp, S, df.R) : estep_s2_scratch_bytes(fgrp, S);
        const int grid2 = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::min<int>(G2, (int)k), SCRATCH_MAX / per2));
        if ((e = scratch_ensure(d_scr2, per2 * grid2, false, true))) return hipfail(e, "estep pass-2 scratch");
        if ((rc = ensure_store(d_trace, std::max<uint64_t>(t, 1), trace_budget, "trace store"))) return rc;
        ValueArgs v;
        v.S = S;
        v.L = L;
        v.head_len = head_len;
        v.order = d_order2.p;
        v.n_order = (int)k;
        v.rec = d_rec.p;
        v.rec_off = d_rec_off.p;
        v.scratch = d_scr2.p;
        v.scratch_stride = per2;
        v.fcap = fgrp;
        v.lds_fc = use_df ? df.fc : s2_tier(S, vnw, vipc, pair);
        v.trace = d_trace.p;
        v.trace_cap = d_trace.n;
        v.trace_cursor = d_trace_cursor.p;
        v.trace_base = d_tbase.p;
        v.loc_off = d_loc_off.p;
        v.status = d_status.p;
        v.total = d_total.p;
        v.ncand = d_ncand.p;
        v.cand_state = d_cstate.p;
        v.cand_idx = d_cidx.p;
        v.prior = d_prior.p;
        v.posterior = d_post.p;
        v.weight = d_weight.p;
        v.cost = d_cost.p;
        v.stamps = d_stamps.p;
        v.next_q = d_nextq.p + 1;
        if ((e = hipMemsetAsync(d_nextq.p + 1, 0, 4, st))) return hipfail(e, "estep");
        const bool fast = value_fast && S <= 32;  // lists longer than a wavefront: exact order only
        hipEventRecord(ev[0], st);
        if (use_df) {
          if ((e = launch_estep_values_df(v, grid2, vnw, vwpe, pair, df.R, df.qcap, st)))
            return hipfail(e, "estep_values_df launch");
        } else if ((e = launch_estep_values(v, grid2, vnw, fast, vwpe, st, pair))) {
          return hipfail(e, "estep_values launch");
        }
        last_value_df = use_df;
        hipEventRecord(ev[1], st);
        if ((rc = read_status(sset, (int)k, true))) return rc;
        hipEventElapsedTime(&ms, ev[0], ev[1]);
        ms_s2 += ms;
        ++n_value_passes;
        if (debug_mem)
          fprintf(stderr, "[hmc] value pass %d: %zu individuals, %.1f ms\n", n_value_passes, k, ms);
        // ---- ties: individuals whose result would depend on the libstdc++ list
        // order re-run on the exact value pass, in their own trace regions
        std::vector<int> h_order;
        for (size_t q = 0; q < k; ++q)
          if (h_status[sset[pos + q]] == EST_NEEDS_ORDER) h_order.push_back(sset[pos + q]);
        n_order_redo += (int)h_order.size();
        if (!h_order.empty()) {
          const int nr = (int)h_order.size();
          if ((e = d_redo.ensure(nr))) return hipfail(e, "estep order re-run");
          if ((rc = upload_order(d_redo, h_order.data(), nr))) return rc;
          ValueArgs v2 = v;
          v2.order = d_redo.p;
          v2.n_order = nr;
          if ((e = hipMemsetAsync(d_nextq.p + 1, 0, 4, st))) return hipfail(e, "estep");
          hipEventRecord(ev[0], st);
          if ((e = launch_estep_values(v2, std::max(1, std::min(G2, nr)), vnw, false, vwpe, st)))
            return hipfail(e, "estep_values launch");
          hipEventRecord(ev[1], st);
          if ((rc = read_status(sset, (int)k, true))) return rc;
          hipEventElapsedTime(&ms, ev[0], ev[1]);
          ms_s2 += ms;
          ms_order += ms;
        }
        h_redo.clear();
        for (size_t q = 0; q < k; ++q) {
          const int bi = sset[pos + q];
          if (h_status[bi] == EST_OVERFLOW_TRACE) return fail(HMC_EHIP, "trace store overflow with exact sizes");
          if (h_status[bi] == EST_NEEDS_ORDER) return fail(HMC_EHIP, "exact value pass reported a tie");
          if (h_status[bi] == EST_DF_STALL) return fail(HMC_EHIP, "dataflow value pass stalled (individual %d)", i0 + bi);
          if (h_status[bi] == EST_NEEDS_EXACT) h_redo.push_back(bi);
        }
        // ---- individuals whose forward likelihood underflowed: the reference
        // skips a pair with fwd <= 0 (extend(), HaploBuilder.cpp:237), which
        // changes their structure.  Their records are rebuilt with that test
        // (structure pass, prune) in their own regions — a subset of the
        // frontiers just walked, so they fit — and their lists re-built.
        n_fallback += (int)h_redo.size();
        if (!h_redo.empty()) {
          const int nr = (int)h_redo.size();
          if ((rc = structure_pass(h_redo.data(), nr, true))) return rc;
          for (int r : h_redo) {
            const int s = h_status[r];
            if (s != EST_OK_PRUNED && s != EST_UNRESOLVED)
              return fail(HMC_EHIP, "underflow re-run: structure status %d (individual %d)", s, i0 + r);
          }
          if ((e = d_redo.ensure(nr))) return hipfail(e, "estep underflow re-run");
          if ((rc = upload_order(d_redo, h_redo.data(), nr))) return rc;
          ValueArgs v2 = v;
          v2.order = d_redo.p;
          v2.n_order = nr;
          if ((e = hipMemsetAsync(d_nextq.p + 1, 0, 4, st))) return hipfail(e, "estep");
          hipEventRecord(ev[0], st);
          if (use_df) {
            if ((e = launch_estep_values_df(v2, std::max(1, std::min(G2, nr)), vnw, vwpe, pair, df.R, df.qcap, st)))
              return hipfail(e, "estep_values_df launch");
          } else if ((e = launch_estep_values(v2, std::max(1, std::min(G2, nr)), vnw, false, vwpe, st, pair))) {
            return hipfail(e, "estep_values launch");
          }
          hipEventRecord(ev[1], st);
          if ((rc = read_status(sset, (int)k, true))) return rc;
          hipEventElapsedTime(&ms, ev[0], ev[1]);
          ms_fb += ms;
          for (int r : h_redo)
            if (h_status[r] != EST_OK && h_status[r] != EST_UNRESOLVED)
              return fail(HMC_EHIP, "underflow re-run: value status %d (individual %d)", h_status[r], i0 + r);
        }
        if ((rc = traceback_group((int)k))) return rc;
        pos += k;
      }
      pending.swap(rest);
    }
    if (!exact) {
      prev_rneed = rneed;
      prev_P = P;
    }
    return HMC_OK;
  }

  // PatternManager::checkFrequency (PatternManager.cpp:146-193) of n given
  // candidates of one length against the current items (genotypes while no
  // samples exist, else the weighted samples): the per-level seam of the
  // reference's DFS (searchPattern, :100-144).  Sums in item order; across
  // ranks in rank order (or one all-reduce), as the mining levels.
  DevBuf<int32_t> d_lv_start;
  DevBuf<uint8_t> d_lv_al;
  DevBuf<double> d_lv_sum;
  int mine_level(int level, int n, const int32_t *start, const int32_t *alleles, double *freq, uint64_t *scanned) {
    if (!have_panel) return fail(HMC_EARG, "no genotypes loaded");
    if (level < 0 || n < 0 || (n > 0 && (!start || !freq || (level > 0 && !alleles))))
      return fail(HMC_EARG, "mine_level arguments");
    const int L = pan.L;
    if (scanned) *scanned = 0;
    if (n == 0) return HMC_OK;
    if (level == 0) {  // HaploPattern of length 0: frequency 1 (checkFrequency :149-150)
      for (int c = 0; c < n; ++c) freq[c] = 1.0;
      return HMC_OK;
    }
    std::vector<uint8_t> al((size_t)n * level);
    for (int c = 0; c < n; ++c) {
      if (start[c] < 0 || start[c] + level > L) return fail(HMC_EARG, "candidate %d outside the loci", c);
      for (int j = 0; j < level; ++j) {
        const auto &sy = pan.sym[start[c] + j];
        const int32_t a = alleles[(size_t)c * level + j];
        uint8_t ix = 0xFD;  // a symbol the locus does not have: matches only missing alleles
        for (size_t q = 0; q < sy.size(); ++q)
          if (sy[q].first == a) ix = (uint8_t)q;
        al[(size_t)c * level + j] = ix;
      }
    }
    hipError_t e;
    if ((e = d_lv_start.ensure(n)) || (e = d_lv_al.ensure(al.size())) || (e = d_lv_sum.ensure(n)) ||
        (e = hipMemcpyAsync(d_lv_start.p, start, (size_t)n * 4, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(d_lv_al.p, al.data(), al.size(), hipMemcpyHostToDevice, st)))
      return hipfail(e, "mine_level");
    const bool genotype = !have_samples;
    MineArgs a = mine_args(genotype);
    int rc;
    if (multi() && reduction == RED_ORDERED) {
      for (int r = 0; r < world; ++r) {
        if (r == rank) {
          a.seeded = r > 0;
          if ((e = launch_mine_scan(a, level, n, d_lv_start.p, d_lv_al.p, d_lv_sum.p, st))) return hipfail(e, "mine_scan");
        }
        if ((rc = bcast(d_lv_sum.p, n, r))) return rc;
      }
    } else {
      if ((e = launch_mine_scan(a, level, n, d_lv_start.p, d_lv_al.p, d_lv_sum.p, st))) return hipfail(e, "mine_scan");
      if ((rc = allreduce_sum(d_lv_sum.p, n))) return rc;
    }
    if ((e = hipMemcpyAsync(freq, d_lv_sum.p, (size_t)n * 8, hipMemcpyDeviceToHost, st)) || (e = hipStreamSynchronize(st)))
      return hipfail(e, "mine_level");
    const double denom = genotype ? (double)pan.N : total_weight;  // :178, :190
    for (int c = 0; c < n; ++c) freq[c] = freq[c] / denom;
    if (scanned) *scanned = (uint64_t)n * (uint64_t)a.n_items;
    return HMC_OK;
  }

  // LDS tiers of pass 1 (one wave per individual, `budget` bytes): states per
  // frontier, key slots (2x, power of two), contributions per locus (2x).
  static void s1_tier(int budget, int amax, int nw, int &fc, int &hc, int &cc) {
    for (int f = 2048; f >= 16; f -= 16) {
      const int h = next_pow2(2 * f), c = 2 * f;
      if ((int)estep_s1_lds_bytes(f, h, c, amax, nw) <= budget) { fc = f; hc = h; cc = c; return; }
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
  bool last_value_df = false;
  struct DfShape {
    int nw = 0, ipc = 0, R = 3, qcap = 64, fc = 0;
  };
  bool df_auto(bool heavy) const { (void)heavy; return false; }
  bool df_shape(int S, bool pair, bool heavy, bool small_heavy, int per_cu, int fgrp, DfShape &d) const {
    d.nw = vp_nw > 0 ? std::max(2, vp_nw) : (small_heavy ? std::max(2, 16 / per_cu) : (heavy ? 8 : 2));
    d.ipc = vp_ipc > 0 ? vp_ipc : (small_heavy ? per_cu : (heavy ? 2 : 8));
    if (d.nw * d.ipc > 20) d.ipc = std::max(1, 20 / d.nw);
    d.R = df_ring;
    const int G = pair ? WAVE / S : WAVE / (2 * S);
    const int nseg = (d.nw - 1) * G;
    d.qcap = 64;
    while (d.qcap < std::max(4 * nseg, heavy ? 512 : 64)) d.qcap *= 2;
    const int budget = 160 * 1024 / std::max(1, d.ipc) - 256;
    if ((int)estep_df_lds_bytes(S, 0, d.nw, pair, d.R, d.qcap, fgrp) > budget) return false;
    int lo = 0, hi = fgrp;  // largest LDS tier that fits
    while (lo < hi) {
      const int mid = (lo + hi + 1) / 2;
      if ((int)estep_df_lds_bytes(S, mid, d.nw, pair, d.R, d.qcap, fgrp) <= budget) lo = mid;
      else hi = mid - 1;
    }
    d.fc = lo;
    return true;
  }

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

  DevModel dev_model() const {
    DevModel m;
    m.P = P;
    m.succ = t_succ.p;
    m.tp = t_tp.p;
    m.freq = t_freq.p;
    m.last = t_last.p;
    m.n_head = n_head;
    m.head_len = head_len;
    m.head_ids = d_head_ids.p;
    m.head_pat0 = d_head_pat0.p;
    if (head_len > 1) {
      m.hf_base = i0;
      m.hf_off = d_hf_off.p;
      m.hf_pairs = d_hf_pairs.p;
      m.hf_status = d_hf_status.p;
      m.head_al = d_head_al.p;
    }
    return m;
  }

  // selected pairs of the last E-step, allele indices [n][2][L]
  int resolutions_idx(std::vector<uint8_t> &out) {
    if (!have_estep) return fail(HMC_EARG, "no E-step has run");
    const int n = nloc(), L = pan.L;
    hipError_t e;
    if ((e = d_res.ensure((size_t)n * 2 * L))) return hipfail(e, "resolutions");
    if ((e = launch_gather_resolutions(d_rows.p, L, d_sbase.p, d_ncand.p, d_geno_im.p, i0, n, d_res.p, st)))
      return hipfail(e, "resolutions");
    out.resize((size_t)n * 2 * L);
    if ((e = hipMemcpyAsync(out.data(), d_res.p, out.size(), hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "resolutions");
    return HMC_OK;
  }

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
  int haplocomp(double out[3]) {
    const int n = nloc(), L = pan.L;
    const int ncmp = std::max(0, std::min(n, pan.unphased - i0));  // m_genotype_num = unphased_num() (HaploComp.cpp:40)
    hipError_t e;
    std::vector<int32_t> hc((size_t)ncmp * 6), bad(ncmp);
    if (ncmp > 0) {
      if ((e = d_hc_cnt.ensure((size_t)ncmp * 6)) || (e = d_hc_bad.ensure(ncmp)) ||
          (e = launch_haplocomp_counts(d_geno_im.p, i0, ncmp, L, d_best.p, d_hc_cnt.p, d_hc_bad.p, st)) ||
          (e = hipMemcpyAsync(hc.data(), d_hc_cnt.p, hc.size() * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipMemcpyAsync(bad.data(), d_hc_bad.p, bad.size() * 4, hipMemcpyDeviceToHost, st)) ||
          (e = hipStreamSynchronize(st)))
        return hipfail(e, "haplocomp");
    }
    double cnt[6] = {0, 0, 0, 0, 0, 0};  // se_num, se_den, ihp_num, ihp_den, igp_num, igp_den
    for (int i = 0; i < ncmp; ++i) {
      if (bad[i] >= 0) return fail(HMC_EARG, "Inconsistent genotypes at locus %d!", bad[i]);
      const int32_t *c = hc.data() + (size_t)i * 6;
      const int sd = c[0], het = c[1];
      cnt[0] += sd;
      cnt[1] += het - 1;
      cnt[2] += sd > 0 ? 1 : 0;
      cnt[3] += het > 1 ? 1 : 0;
      cnt[4] += c[4];
      cnt[5] += c[5];
    }
    int rc = allreduce_host(cnt, 6);  // integers < 2^53: exact in any order
    if (rc) return rc;
    out[0] = cnt[0] / cnt[1];
    out[1] = cnt[2] / cnt[3];
    out[2] = cnt[4] / cnt[5];
    return HMC_OK;
  }

  // the accepted resolutions on the host (outputs)
  int sync_best() {
    if (best_on_host) return HMC_OK;
    hipError_t e;
    best_res.resize((size_t)nloc() * 2 * pan.L);
    if ((e = hipMemcpyAsync(best_res.data(), d_best.p, best_res.size(), hipMemcpyDeviceToHost, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "resolutions");
    best_on_host = true;
    return HMC_OK;
  }

  // ------------------------------------------------------------------ run --
  // resolutions = unphased (HaploModel.cpp:127)
  int init_best() {
    const int n = nloc(), L = pan.L;
    best_res.assign((size_t)n * 2 * L, 0);
    for (int i = 0; i < n; ++i)
      for (int h = 0; h < 2; ++h)
        for (int k = 0; k < L; ++k)
          best_res[((size_t)i * 2 + h) * L + k] = pan.idx[((size_t)(i0 + i) * 2 + h) * L + k];
    hipError_t e;
    if ((e = d_best.ensure(best_res.size())) ||
        (e = hipMemcpyAsync(d_best.p, best_res.data(), best_res.size(), hipMemcpyHostToDevice, st)) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "resolutions");
    have_best = best_on_host = true;
    return HMC_OK;
  }
  // HaploModel.cpp:132-133: resolutions = this E-step's best pairs (device copy)
  int accept_resolutions() {
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
  int em_iteration(int it, int max_iter, bool force_m, double &old_ll, hmc_iter_log &rec, bool &go) {
    using clk = std::chrono::steady_clock;
    int rc;
    if (!have_best && (rc = init_best())) return rc;
    auto t1 = clk::now();
    double ll = 0;
    int Hs = 0;
    uint64_t re = 0;
    if ((rc = estep(&ll, &Hs, &re))) return rc;
    const double te = std::chrono::duration<double>(clk::now() - t1).count();
    if (ll >= old_ll && (rc = accept_resolutions())) return rc;
    rec = hmc_iter_log{};
    double hc[3];
    if ((rc = haplocomp(hc))) return rc;  // HaploModel.cpp:134-136
    rec.switch_error = hc[0];
    rec.ihp = hc[1];
    rec.igp = hc[2];
    rec.log_likelihood = ll;
    rec.t_estep_s = te;
    rec.r_e = re;
    rec.n_samples = Hs;
    rec.n_patterns = P;
    go = it < max_iter && ll >= old_ll && (old_ll - ll) / old_ll > 0.0001;  // HaploModel.cpp:139
    if (go || force_m) {
      auto t2 = clk::now();
      int np = 0;
      uint64_t rm = 0;
      if ((rc = mine(&np, &rm))) return rc;
      rec.t_mstep_s = std::chrono::duration<double>(clk::now() - t2).count();
      rec.r_m = rm;
      rec.n_patterns = np;
      old_ll = ll;
    }
    return HMC_OK;
  }

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
  int model_save() {
    if (!have_model) return fail(HMC_EARG, "no pattern model to save");
    const size_t p = (size_t)std::max(P, 1), A = (size_t)pan.amax;
    // a table over 8 GB (cfg 4's M0: 720 M patterns, 35 GB) is kept in pinned
    // host memory: HBM is the E-step stores'; a rewind then reads it over PCIe
    const bool on_host = (double)p * (41.0 + 4.0 * (double)A) > 8e9;
    snap.start.set_host(on_host);
    snap.len.set_host(on_host);
    snap.node.set_host(on_host);
    snap.ppat.set_host(on_host);
    snap.freq.set_host(on_host);
    snap.prefix.set_host(on_host);
    snap.tp.set_host(on_host);
    snap.last.set_host(on_host);
    snap.succ.set_host(on_host);
    hipError_t e;
    if ((e = dcopy(snap.start, t_start, p)) || (e = dcopy(snap.len, t_len, p)) || (e = dcopy(snap.node, t_node, p)) ||
        (e = dcopy(snap.ppat, t_ppat, p)) ||
        (e = dcopy(snap.freq, t_freq, p)) || (e = dcopy(snap.prefix, t_prefix, p)) || (e = dcopy(snap.tp, t_tp, p)) ||
        (e = dcopy(snap.last, t_last, p)) || (e = dcopy(snap.succ, t_succ, p * A)) ||
        (e = dcopy(snap.head_ids, d_head_ids, std::max<size_t>(n_head, 1))) ||
        (e = dcopy(snap.head_pat0, d_head_pat0, A + 1)) ||
        (head_len > 1 && (e = dcopy(snap.head_al, d_head_al, p * head_len))) || (e = hipStreamSynchronize(st)))
      return hipfail(e, "model_save");
    snap.P = P;
    snap.L = pan.L;
    snap.amax = pan.amax;
    snap.head_len = head_len;
    snap.n_head = n_head;
    snap.gen = model_gen;
    snap.h_head_ids = h_head_ids;
    snap.h_head_al = h_head_al;
    snap.table_on_host = table_on_host;
    if (table_on_host) {
      snap.ht = ht;
      snap.ht_succ = ht_succ;
    }
    snap.valid = true;
    return HMC_OK;
  }
  int em_rewind() {
    if (!snap.valid) return fail(HMC_EARG, "no saved model (hmc_model_save)");
    if (!have_panel || snap.L != pan.L || snap.amax != pan.amax)
      return fail(HMC_EARG, "the saved model belongs to another panel");
    const size_t p = (size_t)std::max(snap.P, 1), A = (size_t)pan.amax;
    hipError_t e;
    if ((e = dcopy(t_start, snap.start, p)) || (e = dcopy(t_len, snap.len, p)) || (e = dcopy(t_node, snap.node, p)) ||
        (e = dcopy(t_ppat, snap.ppat, p)) ||
        (e = dcopy(t_freq, snap.freq, p)) || (e = dcopy(t_prefix, snap.prefix, p)) || (e = dcopy(t_tp, snap.tp, p)) ||
        (e = dcopy(t_last, snap.last, p)) || (e = dcopy(t_succ, snap.succ, p * A)) ||
        (e = dcopy(d_head_ids, snap.head_ids, std::max<size_t>(snap.n_head, 1))) ||
        (e = dcopy(d_head_pat0, snap.head_pat0, A + 1)) ||
        (snap.head_len > 1 && (e = dcopy(d_head_al, snap.head_al, p * snap.head_len))) ||
        (e = hipStreamSynchronize(st)))
      return hipfail(e, "em_rewind");
    P = snap.P;
    head_len = snap.head_len;
    n_head = snap.n_head;
    model_gen = snap.gen;  // the candidate tree is valid again only if nothing was mined since
    h_head_ids = snap.h_head_ids;
    h_head_al = snap.h_head_al;
    table_on_host = snap.table_on_host;
    if (table_on_host) {
      ht = snap.ht;
      ht_succ = snap.ht_succ;
    }
    have_model = true;
    hf_valid = false;
    // the EM state of a fresh HaploModel::run after this M-step
    have_samples = have_estep = have_best = best_on_host = false;
    H = 0;
    total_weight = 0.0;
    h_cost.clear();
    prev_rneed.clear();
    prev_P = 0;
    fcap = fcap_user;
    return HMC_OK;
  }

  int run(int max_iter, hmc_iter_log *log, int cap, int *iters, double *t_m0, uint64_t *rm0, int *np0) {
    using clk = std::chrono::steady_clock;
    have_samples = false;  // HaploModel::build -> setGenoData clears samples (HaploBuilder.cpp:19-23)
    auto t0 = clk::now();
    int np = 0;
    uint64_t rm = 0;
    int rc = mine(&np, &rm);
    if (rc) return rc;
    if (t_m0) *t_m0 = std::chrono::duration<double>(clk::now() - t0).count();
    if (rm0) *rm0 = rm;
    if (np0) *np0 = np;
    if ((rc = init_best())) return rc;
    double old_ll = -DBL_MAX;
    int it = 0;
    for (it = 1; it <= max_iter; ++it) {
      hmc_iter_log rec{};
      bool go = false;
      if ((rc = em_iteration(it, max_iter, false, old_ll, rec, go))) return rc;
      if (log && it - 1 < cap) log[it - 1] = rec;
      if (!go) break;
    }
    if (iters) *iters = std::min(it, max_iter);
    return HMC_OK;
  }
};

}  // namespace hmc

using hmc::Ctx;

struct hmc_ctx {
  Ctx c;
};

// ===================================================================== C-ABI
extern "C" {

const char *hmc_version(void) { return "hmc_amd 0.1 (gfx950)"; }

static int ctx_init(hmc_ctx *h, int device) {
  hipError_t e = hipSetDevice(device);
  if (e) return h->c.hipfail(e, "hipSetDevice");
  h->c.device = device;
  h->c.debug_mem = getenv("HMC_DEBUG_MEM") != nullptr;
  h->c.diag_mine = getenv("HMC_DIAG_MINE") != nullptr;
  if ((e = hipStreamCreateWithFlags(&h->c.st, hipStreamNonBlocking))) return h->c.hipfail(e, "hipStreamCreate");
  for (auto &ev : h->c.ev)
    if ((e = hipEventCreate(&ev))) return h->c.hipfail(e, "hipEventCreate");
  return HMC_OK;
}

int hmc_ctx_create(int device, hmc_ctx **out) {
  if (!out) return HMC_EARG;
  hmc_ctx *h = new hmc_ctx;
  int rc = ctx_init(h, device);
  *out = h;  // returned even on failure so the caller can read hmc_ctx_error
  return rc;
}

int hmc_rccl_unique_id(void *out128) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return HMC_ERCCL;
  memcpy(out128, &id, sizeof id);
  return HMC_OK;
}

int hmc_ctx_create_dist(int device, int rank, int world, const void *unique_id, hmc_ctx **out) {
  if (!out || world < 1 || rank < 0 || rank >= world) return HMC_EARG;
  hmc_ctx *h = new hmc_ctx;
  *out = h;
  int rc = ctx_init(h, device);
  if (rc) return rc;
  h->c.rank = rank;
  h->c.world = world;
  {  // a unique id means an RCCL communicator, also at world 1 (hmc_set_force_collectives)
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof id);
    ncclResult_t r = ncclCommInitRank(&h->c.comm, world, id, rank);
    if (r != ncclSuccess) return h->c.fail(HMC_ERCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  return HMC_OK;
}

int hmc_ctx_create_comm(int device, void *rccl_comm, hmc_ctx **out) {
  if (!out || !rccl_comm) return HMC_EARG;
  hmc_ctx *h = new hmc_ctx;
  *out = h;
  int rc = ctx_init(h, device);
  if (rc) return rc;
  ncclComm_t comm = (ncclComm_t)rccl_comm;
  int r = 0, w = 1;
  if (ncclCommUserRank(comm, &r) != ncclSuccess || ncclCommCount(comm, &w) != ncclSuccess)
    return h->c.fail(HMC_ERCCL, "not an RCCL communicator");
  h->c.comm = comm;
  h->c.own_comm = false;
  h->c.rank = r;
  h->c.world = w;
  return HMC_OK;
}

int hmc_set_force_collectives(hmc_ctx *h, int on) {
  if (!h) return HMC_EARG;
  hmc::Ctx &c = h->c;
  if (on && c.world == 1 && !c.comm && !c.host_fn)
    return c.fail(HMC_EARG, "force_collectives: the context has no communicator (create it with a unique id or a comm)");
  c.force_coll = on != 0 && c.world == 1;
  return HMC_OK;
}

int hmc_rccl_comm_init(int device, int world, int rank, const void *unique_id, void **comm) {
  if (!comm || !unique_id || world < 1 || rank < 0 || rank >= world) return HMC_EARG;
  if (hipSetDevice(device) != hipSuccess) return HMC_EHIP;
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof id);
  ncclComm_t c = nullptr;
  if (ncclCommInitRank(&c, world, id, rank) != ncclSuccess) return HMC_ERCCL;
  *comm = c;
  return HMC_OK;
}

int hmc_rccl_comm_destroy(void *comm) {
  if (!comm) return HMC_EARG;
  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? HMC_OK : HMC_ERCCL;
}

int hmc_set_reduction(hmc_ctx *h, int mode) {
  if (!h || mode < 0 || mode > 1) return HMC_EARG;
  h->c.reduction = mode;
  return HMC_OK;
}

int hmc_ctx_create_hostcoll(int device, int rank, int world, hmc_allreduce_fn fn, void *user, hmc_ctx **out) {
  if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !fn)) return HMC_EARG;
  hmc_ctx *h = new hmc_ctx;
  *out = h;
  int rc = ctx_init(h, device);
  if (rc) return rc;
  h->c.rank = rank;
  h->c.world = world;
  h->c.host_fn = fn;
  h->c.host_user = user;
  return HMC_OK;
}

void hmc_ctx_destroy(hmc_ctx *h) {
  if (!h) return;
  if (h->c.comm && h->c.own_comm) ncclCommDestroy(h->c.comm);
  for (auto &ev : h->c.ev)
    if (ev) hipEventDestroy(ev);
  if (h->c.st) hipStreamDestroy(h->c.st);
  delete h;
}

const char *hmc_ctx_error(const hmc_ctx *h) { return h ? h->c.err.c_str() : "null context"; }

int hmc_set_num_patterns(hmc_ctx *h, int num_patterns) {
  if (!h) return HMC_EARG;
  h->c.num_patterns = num_patterns;
  return HMC_OK;
}

int hmc_set_model(hmc_ctx *h, const char *model, int mc_order) {
  if (!h || !model) return HMC_EARG;
  const std::string m(model);
  if (m == "MV") h->c.model = 0;
  else if (m == "MC") h->c.model = 1;
  else if (m == "MA") h->c.model = 2;
  else return h->c.fail(HMC_EARG, "Unknown model %s!", model);  // HaploModel.cpp:33-34
  if (mc_order < 0) return h->c.fail(HMC_EARG, "mc_order must be >= 0");
  h->c.mc_order = mc_order;
  return HMC_OK;
}

int hmc_set_params(hmc_ctx *h, double min_freq_abs, double min_freq, int min_len, int max_len, int sample_size) {
  if (!h) return HMC_EARG;
  h->c.min_freq_abs = min_freq_abs;
  h->c.min_freq = min_freq;
  h->c.min_len = min_len;
  h->c.max_len = max_len;
  h->c.sample_size = sample_size;
  return HMC_OK;
}

int hmc_set_tuning(hmc_ctx *h, int frontier_cap, uint64_t trace_bytes, int waves) {
  if (!h) return HMC_EARG;
  if (waves < 0) { h->c.lds_waves_per_cu = -waves; waves = 0; }  // negative: E-step waves per CU (LDS split)
  if (frontier_cap > 0) {
    h->c.fcap = h->c.fcap_user = std::min(frontier_cap, hmc::F_MAX);
    h->c.fcap_user_set = true;
  }
  h->c.trace_bytes = trace_bytes;
  h->c.waves = waves;
  return HMC_OK;
}

int hmc_shard_range(const hmc_ctx *h, int *i0, int *i1) {
  if (!h || !i0 || !i1) return HMC_EARG;
  *i0 = h->c.i0;
  *i1 = h->c.i1;
  return HMC_OK;
}

int hmc_set_estep_mode(hmc_ctx *h, int mode) {
  if (!h || mode < 0 || mode > 1) return HMC_EARG;
  h->c.estep_mode = mode;
  return HMC_OK;
}

int hmc_last_estep_split(const hmc_ctx *h, double *structure_ms, double *values_ms, double *fallback_ms,
                         int *n_fallback) {
  if (!h) return HMC_EARG;
  if (structure_ms) *structure_ms = h->c.ms_s1;
  if (values_ms) *values_ms = h->c.ms_s2;
  if (fallback_ms) *fallback_ms = h->c.ms_fb;
  if (n_fallback) *n_fallback = h->c.n_fallback;
  return HMC_OK;
}

int hmc_set_exact_estimate(hmc_ctx *h, int on) {
  if (!h) return HMC_EARG;
  h->c.exact_estimate = on != 0;
  return HMC_OK;
}

int hmc_last_exact_stats(const hmc_ctx *h, int *rounds, uint64_t *candidates, double *walk_ms) {
  if (!h) return HMC_EARG;
  if (rounds) *rounds = h->c.exact_rounds;
  if (candidates) *candidates = h->c.exact_candidates;
  if (walk_ms) *walk_ms = h->c.ms_walk;
  return HMC_OK;
}

int hmc_set_value_mode(hmc_ctx *h, int mode) {
  if (!h || mode < 0 || mode > 1) return HMC_EARG;  // 0: value-only + re-runs, 1: libstdc++ permutations
  h->c.value_fast = mode == 0;
  return HMC_OK;
}

int hmc_set_value_pass(hmc_ctx *h, int mode, int ring) {
  if (!h || mode < 0 || mode > 2 || ring < 0 || ring == 1 || ring == 2 || ring > 4) return HMC_EARG;
  h->c.value_pass = mode;  // 0 automatic, 1 locus-synchronous (estep_values), 2 dataflow (estep_values_df)
  h->c.df_ring = ring ? ring : 3;
  return HMC_OK;
}

int hmc_last_value_pass(const hmc_ctx *h, int *dataflow) {
  if (!h) return HMC_EARG;
  if (dataflow) *dataflow = h->c.last_value_df ? 1 : 0;
  return HMC_OK;
}

int hmc_set_value_layout(hmc_ctx *h, int mode) {
  if (!h || mode < 0 || mode > 2) return HMC_EARG;  // 0 never, 1 heavy groups, 2 every group
  h->c.value_pair = mode;
  return HMC_OK;
}

int hmc_last_estep_order(const hmc_ctx *h, int *n_rerun, double *rerun_ms) {
  if (!h) return HMC_EARG;
  if (n_rerun) *n_rerun = h->c.n_order_redo;
  if (rerun_ms) *rerun_ms = h->c.ms_order;
  return HMC_OK;
}

int hmc_last_estep_passes(const hmc_ctx *h, int *structure_passes, int *value_passes) {
  if (!h) return HMC_EARG;
  if (structure_passes) *structure_passes = h->c.n_struct_passes;
  if (value_passes) *value_passes = h->c.n_value_passes;
  return HMC_OK;
}

int hmc_set_estep_shape(hmc_ctx *h, int waves_per_individual, int individuals_per_cu) {
  if (!h) return HMC_EARG;
  if (waves_per_individual < 0 || waves_per_individual > 4 || individuals_per_cu < 0) return HMC_EARG;
  if (waves_per_individual > 0) h->c.estep_nw = h->c.vp_nw = waves_per_individual;
  if (individuals_per_cu > 0) h->c.lds_waves_per_cu = h->c.vp_ipc = individuals_per_cu;
  if (waves_per_individual == 0 && individuals_per_cu == 0) h->c.vp_nw = h->c.vp_ipc = 0;  // value pass by group size
  return HMC_OK;
}

int hmc_set_pass_shapes(hmc_ctx *h, int structure_waves, int structure_ipc, int value_waves, int value_ipc) {
  if (!h || (structure_waves != 0 && structure_waves != 1 && structure_waves != 4 && structure_waves != 8 &&
             structure_waves != 16) ||
      structure_ipc < 0 ||
      structure_ipc > 32 || value_waves < 0 || value_waves > 16 || value_ipc < 0 || value_ipc > 32)
    return HMC_EARG;
  h->c.s1_nw = structure_waves;
  h->c.s1_ipc = structure_ipc;
  h->c.vp_nw = value_waves;
  h->c.vp_ipc = value_ipc;
  return HMC_OK;
}

int hmc_set_store_budgets(hmc_ctx *h, uint64_t trace_bytes, uint64_t record_bytes) {
  if (!h) return HMC_EARG;
  h->c.trace_bytes = trace_bytes;
  h->c.rec_bytes = record_bytes;
  return HMC_OK;
}

int hmc_set_mine_block(hmc_ctx *h, int start_loci) {
  if (!h || start_loci < 0) return HMC_EARG;
  h->c.mine_block_starts = start_loci;
  return HMC_OK;
}

int hmc_last_estep_frontier(hmc_ctx *h, int *max_states, int *frontier_cap) {
  if (!h) return HMC_EARG;
  uint32_t m = 0;
  if (h->c.d_maxst.p) {
    hipError_t e = hipMemcpy(&m, h->c.d_maxst.p, 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return h->c.hipfail(e, "frontier stats");
  }
  if (max_states) *max_states = (int)m;
  if (frontier_cap) *frontier_cap = h->c.fcap;
  return HMC_OK;
}

int hmc_set_mine_memory(hmc_ctx *h, uint64_t list_bytes) {
  if (!h) return HMC_EARG;
  h->c.mine_list_cap = list_bytes;
  return HMC_OK;
}

int hmc_last_mine_stats(const hmc_ctx *h, int *blocks, int64_t *nodes, double *node_window_gb) {
  if (!h) return HMC_EARG;
  if (blocks) *blocks = h->c.last_mine_blocks;
  if (nodes) *nodes = h->c.last_mine_nodes;
  if (node_window_gb) *node_window_gb = h->c.last_mine_window_gb;
  return HMC_OK;
}

int hmc_model_save(hmc_ctx *h) { return h ? h->c.model_save() : HMC_EARG; }
int hmc_em_rewind(hmc_ctx *h) { return h ? h->c.em_rewind() : HMC_EARG; }

const char *hmc_build_info(void) {
  return "hmc_amd 0.3 gfx950 -O3 -ffp-contract=off, built " __DATE__ " " __TIME__;
}

int hmc_load_phase(hmc_ctx *h, const char *path) {
  if (!h || !path) return HMC_EARG;
  hmc::Panel p;
  hmc::FileData meta;
  std::string err;
  if (!hmc::read_phase(path, p, meta, err)) return h->c.fail(HMC_EIO, "%s", err.c_str());
  h->c.pan = std::move(p);
  h->c.file_meta = std::move(meta);
  return h->c.upload_panel();
}

int hmc_load_genotypes(hmc_ctx *h, int N, int L, const int32_t *alleles, const char *types) {
  if (!h || N <= 0 || L <= 0 || !alleles) return HMC_EARG;
  hmc::Panel p;
  p.N = N;
  p.L = L;
  p.al.assign(alleles, alleles + (size_t)N * 2 * L);
  p.types = types ? std::string(types, strnlen(types, (size_t)L)) : std::string(L, 'S');
  if ((int)p.types.size() < L) p.types.resize(L, 'S');
  std::string err;
  if (!p.build_tables(err)) return h->c.fail(HMC_EUNSUPPORTED, "%s", err.c_str());
  h->c.pan = std::move(p);
  h->c.file_meta = hmc::FileData();  // no ids / positions: writers use the defaults
  return h->c.upload_panel();
}

static std::vector<std::string> path_list(const char *const *paths, int n) {
  std::vector<std::string> v;
  for (int i = 0; i < n; ++i) v.push_back(paths[i] ? paths[i] : "");
  return v;
}

// Any format of HaploFile::getHaploFile (HaploFile.cpp:28-47) into FileData.
static bool parse_any(const char *format, const std::vector<std::string> &paths, hmc::FileData &d, std::string &err) {
  if (std::string(format) == "PHASE") {
    if (paths.empty()) { err = "PHASE needs 1 file name"; return false; }
    hmc::Panel p;
    if (!hmc::read_phase(paths[0].c_str(), p, d, err)) return false;
    d.al = std::move(p.al);
    d.types = p.types;
    return true;
  }
  return hmc::read_geno_file(format, paths, d, err);
}

int hmc_parse_files(const char *format, const char *const *paths, int n_paths, int *N, int *L, int32_t *alleles,
                    char *types, int *unphased) {
  if (!format || !paths || n_paths <= 0) return HMC_EARG;
  hmc::FileData d;
  std::string err;
  if (!parse_any(format, path_list(paths, n_paths), d, err)) return HMC_EIO;
  if (N) *N = d.N;
  if (L) *L = d.L;
  if (unphased) *unphased = d.unphased < 0 ? d.N : d.unphased;
  if (alleles) std::copy(d.al.begin(), d.al.end(), alleles);
  if (types) {
    std::copy(d.types.begin(), d.types.end(), types);
    types[d.L] = 0;
  }
  return HMC_OK;
}

int hmc_parse_file(const char *format, const char *path, const char *path2, int *N, int *L, int32_t *alleles,
                   char *types) {
  if (!path) return HMC_EARG;
  const char *ps[2] = {path, path2};
  return hmc_parse_files(format, ps, path2 ? 2 : 1, N, L, alleles, types, nullptr);
}

int hmc_load_files(hmc_ctx *h, const char *format, const char *const *paths, int n_paths) {
  if (!h || !format || !paths || n_paths <= 0) return HMC_EARG;
  if (std::string(format) == "PHASE") return hmc_load_phase(h, paths[0]);
  hmc::FileData d;
  std::string err;
  if (!hmc::read_geno_file(format, path_list(paths, n_paths), d, err)) return h->c.fail(HMC_EIO, "%s", err.c_str());
  if (d.N <= 0 || d.L <= 0) return h->c.fail(HMC_EIO, "Invalid file type!");
  const int rc = hmc_load_genotypes(h, d.N, d.L, d.al.data(), d.types.c_str());
  if (rc) return rc;
  if (d.unphased >= 0) h->c.pan.unphased = d.unphased;
  h->c.file_meta = std::move(d);
  h->c.file_meta.al.clear();
  return HMC_OK;
}

int hmc_load_file(hmc_ctx *h, const char *format, const char *path, const char *path2) {
  if (!path) return HMC_EARG;
  const char *ps[2] = {path, path2};
  return hmc_load_files(h, format, ps, path2 ? 2 : 1);
}

int hmc_unphased_num(const hmc_ctx *h, int *n) {
  if (!h || !n || !h->c.have_panel) return HMC_EARG;
  *n = h->c.pan.unphased;
  return HMC_OK;
}

// Writer metadata: the loaded file's ids / marker names / positions, or the
// reference's defaults (ids "1".."N", names "M<k+1>", positions k * 1000).
static hmc::FileData writer_meta(const hmc::Ctx &c) {
  hmc::FileData d = c.file_meta;
  d.N = c.pan.N;
  d.L = c.pan.L;
  d.types = c.pan.types;
  if ((int)d.ids.size() != d.N) {
    d.ids.resize(d.N);
    for (int i = 0; i < d.N; ++i) d.ids[i] = std::to_string(i + 1);
  }
  if ((int)d.names.size() != d.L || (int)d.pos.size() != d.L) {
    d.names.resize(d.L);
    d.pos.resize(d.L);
    for (int k = 0; k < d.L; ++k) {
      d.names[k] = "M" + std::to_string(k + 1);
      d.pos[k] = k * 1000;
    }
  }
  return d;
}

int hmc_write_files(hmc_ctx *h, const char *format, const char *const *paths, int n_paths) {
  if (!h || !format || !paths || n_paths <= 0 || !h->c.have_best || h->c.world != 1) return HMC_EARG;
  if (std::string(format) == "PHASE") return hmc_write_phase(h, paths[0]);
  hmc::Ctx &c = h->c;
  if (const int rc = c.sync_best()) return rc;
  const hmc::FileData d = writer_meta(c);
  std::vector<int32_t> hap((size_t)d.N * 2 * d.L);
  c.to_symbols(c.best_res, hap.data());
  std::string err;
  if (!hmc::write_geno_file(format, paths[0], n_paths > 1 ? paths[1] : nullptr, d, hap, err))
    return c.fail(HMC_EIO, "%s", err.c_str());
  return HMC_OK;
}

int hmc_write_file(hmc_ctx *h, const char *format, const char *path, const char *path2) {
  if (!path) return HMC_EARG;
  const char *ps[2] = {path, path2};
  return hmc_write_files(h, format, ps, path2 ? 2 : 1);
}

int hmc_write_patterns(hmc_ctx *h, const char *path) {
  if (!h || !path || !h->c.have_model) return HMC_EARG;
  hmc::Ctx &c = h->c;
  const int P = c.P, L = c.pan.L;
  std::vector<int32_t> st(P), ln(P);
  std::vector<double> fr(P);
  int rc = hmc_get_patterns(h, st.data(), ln.data(), fr.data(), nullptr, nullptr, nullptr, nullptr, 0);
  if (rc) return rc;
  int maxlen = 1;
  for (int i = 0; i < P; ++i) maxlen = std::max(maxlen, ln[i]);
  std::vector<int32_t> al((size_t)P * maxlen);
  if (c.table_on_host) {
    if ((rc = hmc_get_patterns(h, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, al.data(), maxlen))) return rc;
  } else {
    // spelled from the prefix ids (no candidate tree needed: blocked searches
    // and rewound tables qualify); a table whose strings are unknown fails
    // here instead of being written with its last alleles only
    std::vector<int64_t> off;
    std::vector<uint8_t> a8;
    if ((rc = c.spell_table(ln, off, a8))) return rc;
    for (int i = 0; i < P; ++i)
      for (int k = 0; k < ln[i]; ++k) al[(size_t)i * maxlen + k] = c.pan.symbol(st[i] + k, a8[off[i] + k]);
  }
  FILE *fp = fopen(path, "w");
  if (!fp) return c.fail(HMC_EIO, "Can not open file %s!", path);
  fprintf(fp, "Frequency\tLength\t");
  for (int k = 0; k < L; ++k)
    fprintf(fp, "%s ", (int)c.file_meta.names.size() == L ? c.file_meta.names[k].c_str() : ("M" + std::to_string(k + 1)).c_str());
  fprintf(fp, "\n");
  for (int i = 0; i < P; ++i) {  // HaploPattern::write(buf, true): -1 outside [start, end), 'M' integers
    fprintf(fp, "%f\t%d\t", fr[i] / c.pan.N, ln[i]);
    for (int k = 0; k < st[i]; ++k) fprintf(fp, "-1 ");
    for (int k = 0; k < ln[i]; ++k) fprintf(fp, "%d ", al[(size_t)i * maxlen + k]);
    for (int k = st[i] + ln[i]; k < L; ++k) fprintf(fp, "-1 ");
    fprintf(fp, "\n");
  }
  fclose(fp);
  return HMC_OK;
}

int hmc_panel_info(const hmc_ctx *h, int *N, int *L, int *amax) {
  if (!h || !h->c.have_panel) return HMC_EARG;
  if (N) *N = h->c.pan.N;
  if (L) *L = h->c.pan.L;
  if (amax) *amax = h->c.pan.amax;
  return HMC_OK;
}

int hmc_allele_table(const hmc_ctx *h, int32_t *num, int32_t *sym, double *freq) {
  if (!h || !h->c.have_panel) return HMC_EARG;
  const auto &p = h->c.pan;
  for (int k = 0; k < p.L; ++k) {
    if (num) num[k] = (int32_t)p.sym[k].size();
    for (int j = 0; j < p.amax; ++j) {
      const bool ok = j < (int)p.sym[k].size();
      if (sym) sym[(size_t)k * p.amax + j] = ok ? p.sym[k][j].first : -1;
      if (freq) freq[(size_t)k * p.amax + j] = ok ? p.sym[k][j].second : 0.0;
    }
  }
  return HMC_OK;
}

int hmc_find_patterns(hmc_ctx *h, int *n_patterns, uint64_t *r_m) {
  if (!h) return HMC_EARG;
  return h->c.mine(n_patterns, r_m);
}

int hmc_mine_level(hmc_ctx *h, int level, int n, const int32_t *start, const int32_t *alleles, double *freq,
                   uint64_t *scanned) {
  if (!h) return HMC_EARG;
  return h->c.mine_level(level, n, start, alleles, freq, scanned);
}

int hmc_model_info(const hmc_ctx *h, int *n_patterns, int *head_len) {
  if (!h || !h->c.have_model) return HMC_EARG;
  if (n_patterns) *n_patterns = h->c.P;
  if (head_len) *head_len = h->c.head_len;
  return HMC_OK;
}

int hmc_get_patterns(hmc_ctx *h, int32_t *start, int32_t *len, double *freq, double *prefix, double *tp,
                     int32_t *succ, int32_t *alleles, int maxlen) {
  if (!h || !h->c.have_model) return HMC_EARG;
  Ctx &c = h->c;
  const int P = c.P, A = c.pan.amax;
  std::vector<int32_t> st(P), ln(P);
  std::vector<uint8_t> last(P);
  hipError_t e;
  if ((e = hipMemcpyAsync(st.data(), c.t_start.p, (size_t)P * 4, hipMemcpyDeviceToHost, c.st)) ||
      (e = hipMemcpyAsync(ln.data(), c.t_len.p, (size_t)P * 4, hipMemcpyDeviceToHost, c.st)) ||
      (freq && (e = hipMemcpyAsync(freq, c.t_freq.p, (size_t)P * 8, hipMemcpyDeviceToHost, c.st))) ||
      (prefix && (e = hipMemcpyAsync(prefix, c.t_prefix.p, (size_t)P * 8, hipMemcpyDeviceToHost, c.st))) ||
      (tp && (e = hipMemcpyAsync(tp, c.t_tp.p, (size_t)P * 8, hipMemcpyDeviceToHost, c.st))) ||
      (e = hipMemcpyAsync(last.data(), c.t_last.p, (size_t)P, hipMemcpyDeviceToHost, c.st)) ||
      (e = hipStreamSynchronize(c.st)))
    return c.hipfail(e, "get_patterns");
  if (start) memcpy(start, st.data(), (size_t)P * 4);
  if (len) memcpy(len, ln.data(), (size_t)P * 4);
  if (succ) {
    std::vector<uint32_t> s((size_t)P * A);
    if ((e = hipMemcpyAsync(s.data(), c.t_succ.p, s.size() * 4, hipMemcpyDeviceToHost, c.st)) ||
        (e = hipStreamSynchronize(c.st)))
      return c.hipfail(e, "get_patterns");
    for (size_t i = 0; i < s.size(); ++i) succ[i] = s[i] == hmc::NONE ? -1 : (int32_t)s[i];
  }
  if (alleles && maxlen > 0 && c.table_on_host) {  // the exact M-step's table keeps its alleles on the host
    for (int i = 0; i < P; ++i) {
      int32_t *row = alleles + (size_t)i * maxlen;
      for (int k = 0; k < maxlen; ++k) row[k] = k < ln[i] ? c.pan.symbol(st[i] + k, c.ht.alleles(i)[k]) : -1;
    }
  } else if (alleles && maxlen > 0) {
    // allele strings spelled from the prefix ids (or the candidate tree);
    // a table set from outside knows only each pattern's last allele
    std::vector<int64_t> off;
    std::vector<uint8_t> al;
    const bool spelled = c.spell_table(ln, off, al) == HMC_OK;
    if (!spelled) c.err.clear();
    for (int i = 0; i < P; ++i) {
      int32_t *row = alleles + (size_t)i * maxlen;
      for (int k = 0; k < maxlen; ++k) row[k] = -1;
      if (spelled) {
        for (int k = 0; k < ln[i] && k < maxlen; ++k) row[k] = c.pan.symbol(st[i] + k, al[off[i] + k]);
      } else if (ln[i] - 1 < maxlen && ln[i] > 0) {
        row[ln[i] - 1] = c.pan.symbol(st[i] + ln[i] - 1, last[i]);
      }
    }
  }
  return HMC_OK;
}

int hmc_set_patterns(hmc_ctx *h, int P, const int32_t *start, const int32_t *len, const double *freq, const double *tp,
                     const int32_t *succ, const int32_t *last_symbol) {
  if (!h || !h->c.have_panel || P <= 0) return HMC_EARG;
  Ctx &c = h->c;
  const int A = c.pan.amax;
  int rc = c.alloc_table(P);
  if (rc) return rc;
  std::vector<uint8_t> last(P);
  std::vector<uint32_t> s((size_t)P * A);
  std::vector<int32_t> node(P, -1);
  std::vector<std::pair<uint32_t, uint8_t>> heads;
  int hl = std::max(c.min_len, 1);
  for (int i = 0; i < P; ++i) {
    const int k = start[i] + len[i] - 1;
    const int j = c.pan.index_of(k, last_symbol[i]);
    if (j < 0) return c.fail(HMC_EARG, "pattern %d: allele not in locus table", i);
    last[i] = (uint8_t)j;
    for (int a = 0; a < A; ++a) s[(size_t)i * A + a] = succ[(size_t)i * A + a] < 0 ? hmc::NONE : (uint32_t)succ[(size_t)i * A + a];
    if (start[i] == 0 && len[i] == hl) heads.push_back({(uint32_t)i, (uint8_t)j});
  }
  hipError_t e;
  if ((e = hipMemcpyAsync(c.t_start.p, start, (size_t)P * 4, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_len.p, len, (size_t)P * 4, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_node.p, node.data(), (size_t)P * 4, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_freq.p, freq, (size_t)P * 8, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_prefix.p, freq, (size_t)P * 8, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_tp.p, tp, (size_t)P * 8, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_last.p, last.data(), (size_t)P, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemcpyAsync(c.t_succ.p, s.data(), s.size() * 4, hipMemcpyHostToDevice, c.st)) ||
      (e = hipMemsetAsync(c.t_ppat.p, 0xFE, (size_t)P * 4, c.st)) ||  // prefixes unknown
      (e = hipStreamSynchronize(c.st)))
    return c.hipfail(e, "set_patterns");
  c.P = P;
  c.head_len = hl;
  c.table_on_host = false;
  c.h_head_ids.clear();  // head alleles unknown: the E-step supports head_len 1 only here
  c.h_head_al.clear();
  c.new_table(false);  // allele strings are not known for an injected table
  rc = c.set_heads(heads);
  if (rc) return rc;
  c.have_model = true;
  return HMC_OK;
}

int hmc_resolve_all(hmc_ctx *h, double *ll, int *n_samples, uint64_t *r_e) {
  if (!h) return HMC_EARG;
  return h->c.estep(ll, n_samples, r_e);
}

int hmc_get_estep(hmc_ctx *h, double *total, int32_t *ncand, int32_t *status, double *prior, double *posterior,
                  double *weight) {
  if (!h || !h->c.have_estep) return HMC_EARG;
  Ctx &c = h->c;
  const int n = c.nloc(), S = c.S();
  if (total) memcpy(total, c.h_total.data(), (size_t)n * 8);
  if (ncand) memcpy(ncand, c.h_ncand.data(), (size_t)n * 4);
  if (status) memcpy(status, c.h_status.data(), (size_t)n * 4);
  std::vector<double> buf((size_t)n * hmc::S_MAX);
  hipError_t e;
  double *outs[3] = {prior, posterior, weight};
  double *srcs[3] = {c.d_prior.p, c.d_post.p, c.d_weight.p};
  for (int q = 0; q < 3; ++q) {
    if (!outs[q]) continue;
    if ((e = hipMemcpyAsync(buf.data(), srcs[q], buf.size() * 8, hipMemcpyDeviceToHost, c.st)) ||
        (e = hipStreamSynchronize(c.st)))
      return c.hipfail(e, "get_estep");
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < S; ++k)
        outs[q][(size_t)i * S + k] = k < c.h_ncand[i] ? buf[(size_t)i * hmc::S_MAX + k] : 0.0;
  }
  return HMC_OK;
}

int hmc_get_estep_stats(hmc_ctx *h, int32_t *fmax) {
  if (!h || !h->c.have_estep || !fmax) return HMC_EARG;
  hipError_t e;
  if ((e = hipMemcpyAsync(fmax, h->c.d_fmax.p, (size_t)h->c.nloc() * 4, hipMemcpyDeviceToHost, h->c.st)) ||
      (e = hipStreamSynchronize(h->c.st)))
    return h->c.hipfail(e, "get_estep_stats");
  return HMC_OK;
}

int hmc_get_estep_cost(hmc_ctx *h, int32_t *cost) {
  if (!h || !h->c.have_estep || !cost) return HMC_EARG;
  if ((int)h->c.h_cost.size() != h->c.nloc()) return HMC_EARG;
  std::copy(h->c.h_cost.begin(), h->c.h_cost.end(), cost);
  return HMC_OK;
}

int hmc_get_stamps(hmc_ctx *h, uint64_t *out40) {
  if (!h || !out40 || !h->c.d_stamps.p) return HMC_EARG;
  hipError_t e;
  if ((e = hipMemcpyAsync(out40, h->c.d_stamps.p, 40 * 8, hipMemcpyDeviceToHost, h->c.st)) ||
      (e = hipStreamSynchronize(h->c.st)))
    return h->c.hipfail(e, "get_stamps");
  return HMC_OK;
}

int hmc_get_samples(hmc_ctx *h, int32_t *alleles, double *weights, double *total_weight) {
  if (!h || !h->c.have_estep) return HMC_EARG;
  Ctx &c = h->c;
  const int H = c.H, L = c.pan.L;
  hipError_t e;
  if (alleles && H) {  // sample rows live in per-individual slots; h_rowmap gives the sample order
    int32_t top = 0;
    for (int s = 0; s < H; ++s) top = std::max(top, c.h_rowmap[s] + 1);
    std::vector<uint8_t> rows((size_t)top * L);
    if ((e = hipMemcpyAsync(rows.data(), c.d_rows.p, rows.size(), hipMemcpyDeviceToHost, c.st)) ||
        (e = hipStreamSynchronize(c.st)))
      return c.hipfail(e, "get_samples");
    for (int s = 0; s < H; ++s)
      for (int k = 0; k < L; ++k) alleles[(size_t)s * L + k] = c.pan.symbol(k, rows[(size_t)c.h_rowmap[s] * L + k]);
  }
  if (weights && H) {
    if ((e = hipMemcpyAsync(weights, c.d_w.p, (size_t)H * 8, hipMemcpyDeviceToHost, c.st)) ||
        (e = hipStreamSynchronize(c.st)))
      return c.hipfail(e, "get_samples");
  }
  if (total_weight) *total_weight = c.total_weight;
  return HMC_OK;
}

int hmc_get_resolutions(hmc_ctx *h, int32_t *out) {
  if (!h || !out) return HMC_EARG;
  std::vector<uint8_t> idx;
  int rc = h->c.resolutions_idx(idx);
  if (rc) return rc;
  h->c.to_symbols(idx, out);
  return HMC_OK;
}

int hmc_run(hmc_ctx *h, int max_iteration, hmc_iter_log *log, int log_cap, int *iterations, double *t_m0_s,
            uint64_t *r_m0, int *n_patterns0) {
  if (!h) return HMC_EARG;
  return h->c.run(max_iteration, log, log_cap, iterations, t_m0_s, r_m0, n_patterns0);
}

int hmc_clear_samples(hmc_ctx *h) {
  if (!h) return HMC_EARG;
  h->c.have_samples = false;
  h->c.H = 0;
  return HMC_OK;
}

int hmc_em_iteration(hmc_ctx *h, int iteration, int max_iter, int always_mstep, double *old_ll, hmc_iter_log *log,
                     int *go) {
  if (!h || !old_ll) return HMC_EARG;
  if (!h->c.have_model) return h->c.fail(HMC_EARG, "no pattern model: hmc_find_patterns first");
  hmc_iter_log rec{};
  bool g = false;
  const int rc = h->c.em_iteration(iteration, max_iter, always_mstep != 0, *old_ll, rec, g);
  if (rc) return rc;
  if (log) *log = rec;
  if (go) *go = g ? 1 : 0;
  return HMC_OK;
}

int hmc_haplocomp(hmc_ctx *h, double *switch_error, double *ihp, double *igp) {
  if (!h || !h->c.have_best) return HMC_EARG;
  double out[3];
  const int rc = h->c.haplocomp(out);
  if (rc) return rc;
  if (switch_error) *switch_error = out[0];
  if (ihp) *ihp = out[1];
  if (igp) *igp = out[2];
  return HMC_OK;
}

int hmc_get_best_resolutions(hmc_ctx *h, int32_t *out) {
  if (!h || !out || !h->c.have_best) return HMC_EARG;
  if (const int rc = h->c.sync_best()) return rc;
  h->c.to_symbols(h->c.best_res, out);
  return HMC_OK;
}

int hmc_write_phase(hmc_ctx *h, const char *path) {
  if (!h || !path || !h->c.have_best || h->c.world != 1) return HMC_EARG;
  Ctx &c = h->c;
  if (const int rc = c.sync_best()) return rc;
  FILE *fp = fopen(path, "w");
  if (!fp) return c.fail(HMC_EIO, "Can not open file %s!", path);
  const int N = c.pan.N, L = c.pan.L;
  const hmc::FileData d = writer_meta(c);
  fprintf(fp, "%d\n%d\nP", N, L);
  for (int k = 0; k < L; ++k) fprintf(fp, " %d", d.pos[k]);
  fprintf(fp, "\n%s\n", c.pan.types.c_str());
  for (int i = 0; i < N; ++i) {
    const std::string &id = d.ids[i];  // '#' only before an id starting with a digit (HaploFile.cpp:141-147)
    fprintf(fp, (!id.empty() && id[0] >= '0' && id[0] <= '9') ? "#%s\n" : "%s\n", id.c_str());
    for (int hh = 0; hh < 2; ++hh) {
      for (int k = 0; k < L; ++k) {
        const int32_t a = c.pan.symbol(k, c.best_res[((size_t)i * 2 + hh) * L + k]);
        if (c.pan.types[k] == 'S') fprintf(fp, "%c ", a < 0 ? '?' : (char)a);
        else fprintf(fp, "%d ", a);
      }
      fprintf(fp, "\n");
    }
  }
  fclose(fp);
  return HMC_OK;
}

int hmc_last_timings(const hmc_ctx *h, double *f, double *t, double *m) {
  if (!h) return HMC_EARG;
  if (f) *f = h->c.ms_fwd;
  if (t) *t = h->c.ms_tb;
  if (m) *m = h->c.ms_m;
  return HMC_OK;
}

void hmc_test_nth_element(double *lik, uint32_t *tag, int n, int nth) {
  hmc::LinkList v{lik, tag, 1};
  hmc::nth_element_greater(v, n, nth);
}

int hmc_test_coop_nth_element(int device, double *lik, uint32_t *tag, const int32_t *off, const int32_t *n,
                              const int32_t *nth, int count, int total, int seg_width) {
  if (hipSetDevice(device) != hipSuccess) return HMC_EHIP;
  if (seg_width < 2 || seg_width > 32) return HMC_EARG;
  for (int j = 0; j < count; ++j)
    if (n[j] < 0 || n[j] > seg_width || nth[j] < 0 || nth[j] > n[j] || off[j] < 0 || off[j] + n[j] > total)
      return HMC_EARG;
  hmc::DevBuf<double> dl;
  hmc::DevBuf<uint32_t> dt;
  hmc::DevBuf<int32_t> doff, dn, dnth;
  hipError_t e;
  if ((e = dl.ensure(total)) || (e = dt.ensure(total)) || (e = doff.ensure(count)) || (e = dn.ensure(count)) ||
      (e = dnth.ensure(count)))
    return HMC_EHIP;
  if ((e = hipMemcpy(dl.p, lik, (size_t)total * 8, hipMemcpyHostToDevice)) ||
      (e = hipMemcpy(dt.p, tag, (size_t)total * 4, hipMemcpyHostToDevice)) ||
      (e = hipMemcpy(doff.p, off, (size_t)count * 4, hipMemcpyHostToDevice)) ||
      (e = hipMemcpy(dn.p, n, (size_t)count * 4, hipMemcpyHostToDevice)) ||
      (e = hipMemcpy(dnth.p, nth, (size_t)count * 4, hipMemcpyHostToDevice)))
    return HMC_EHIP;
  if ((e = hmc::launch_test_coop_nth(dl.p, dt.p, doff.p, dn.p, dnth.p, count, seg_width, nullptr))) return HMC_EHIP;
  if ((e = hipMemcpy(lik, dl.p, (size_t)total * 8, hipMemcpyDeviceToHost)) ||
      (e = hipMemcpy(tag, dt.p, (size_t)total * 4, hipMemcpyDeviceToHost)))
    return HMC_EHIP;
  return HMC_OK;
}

void hmc_test_nth_element_masks(double *lik, uint32_t *tag, int n, int nth) {
  hmc::LinkList v{lik, tag, 1};
  hmc::nth_element_greater_masks(v, n, nth, n);
}

void hmc_test_sort_small(double *lik, uint32_t *tag, int n) {
  hmc::LinkList v{lik, tag, 1};
  hmc::sort_greater_small(v, n);
}

void hmc_test_sort(double *lik, uint32_t *tag, int n) {
  hmc::LinkList v{lik, tag, 1};
  hmc::sort_greater(v, n);
}

}  // extern "C"
