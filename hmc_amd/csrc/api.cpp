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
#include "ctx.hpp"


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
  h->c.check_records = getenv("HMC_CHECK_RECORDS") != nullptr;
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

int hmc_set_shard(hmc_ctx *h, int i0, int i1) {
  if (!h) return HMC_EARG;
  hmc::Ctx &c = h->c;
  if (!c.have_panel) return c.fail(HMC_EARG, "no panel");
  if (c.world != 1 || i0 < 0 || i1 <= i0 || i1 > c.pan.N)
    return c.fail(HMC_EARG, "shard [%d, %d) of a %d-rank context over %d individuals", i0, i1, c.world, c.pan.N);
  c.i0 = i0;
  c.i1 = i1;
  // nothing learned about the old shard carries over: no samples, no E-step,
  // no accepted resolutions, no per-individual costs or store estimates
  c.have_samples = c.have_estep = c.have_best = c.best_on_host = false;
  c.hf_valid = false;
  c.H = 0;
  c.h_cost.clear();
  c.prev_rneed.clear();
  c.prev_P = 0;
  c.win_scale = 1.0;  // window shrinking learnt on the old shard does not carry over
  return HMC_OK;
}

// The kernels measured slower than the automatic paths (the fused E-step,
// the dataflow value pass, the three-scan structure pass, the four-item exact
// walk) are built into libhmc_amd_variants.so only (make variants); the
// product library refuses to select them.
#ifdef HMC_VARIANTS
static int variant_ok(hmc_ctx *) { return HMC_OK; }
#else
static int variant_ok(hmc_ctx *h) {
  return h->c.fail(HMC_EUNSUPPORTED, "this kernel variant is built into libhmc_amd_variants.so only (make variants)");
}
#endif

int hmc_set_estep_mode(hmc_ctx *h, int mode) {
  if (!h || mode < 0 || mode > 1) return HMC_EARG;
  if (mode == 1 && variant_ok(h)) return HMC_EUNSUPPORTED;
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
  if (!h || mode < 0 || mode > 2) return HMC_EARG;  // 0: value-only + re-runs, 1: libstdc++ permutations, 2: automatic
  h->c.value_mode = mode;
  return HMC_OK;
}

int hmc_set_value_pass(hmc_ctx *h, int mode, int ring) {
  if (!h || mode < 0 || mode > 2 || ring < 0 || ring == 1 || ring == 2 || ring > 4) return HMC_EARG;
  if (mode == 2 && variant_ok(h)) return HMC_EUNSUPPORTED;
  h->c.value_pass = mode;  // 0 automatic, 1 locus-synchronous (estep_values), 2 dataflow (estep_values_df)
  h->c.df_ring = ring ? ring : 3;
  return HMC_OK;
}

int hmc_set_end_order(hmc_ctx *h, int on) {
  if (!h || on < 0 || on > 1) return HMC_EARG;
  h->c.end_order = on != 0;
  return HMC_OK;
}

int hmc_set_dataflow_waves(hmc_ctx *h, int a_waves) {
  if (!h || a_waves < 0 || a_waves > 8) return HMC_EARG;
  h->c.df_na = a_waves;  // 0: by the launch shape
  return HMC_OK;
}

int hmc_set_exact_walk(hmc_ctx *h, int items_per_wave) {
  if (!h || (items_per_wave != 0 && items_per_wave != 1 && items_per_wave != 2 && items_per_wave != 4)) return HMC_EARG;
  if (items_per_wave >= 2 && variant_ok(h)) return HMC_EUNSUPPORTED;
  h->c.exact_ipw = items_per_wave == 0 ? 1 : items_per_wave;
  return HMC_OK;
}

int hmc_set_structure_pass(hmc_ctx *h, int version) {
  if (!h || version < 0 || version > 2) return HMC_EARG;  // 0 = automatic
  if (version == 2 && variant_ok(h)) return HMC_EUNSUPPORTED;
  h->c.structure_pass_version = version == 0 ? 1 : version;
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

int hmc_last_exact_walk(const hmc_ctx *h, int64_t *units, int64_t *launches, int64_t *deferred, int *pruned) {
  if (!h) return HMC_EARG;
  if (units) *units = h->c.xw_units;
  if (launches) *launches = h->c.xw_launches;
  if (deferred) *deferred = h->c.xw_defers;
  if (pruned) *pruned = h->c.exact_pruned;
  return HMC_OK;
}

int hmc_set_estep_windows(hmc_ctx *h, int mode, int window_loci) {
  if (!h || mode < 0 || mode > 2 || window_loci < 0) return HMC_EARG;
  h->c.window_mode = mode;  // 0 automatic, 1 never, 2 always
  h->c.window_loci = window_loci;
  return HMC_OK;
}

int hmc_last_estep_windows(const hmc_ctx *h, int *windows, int *window_loci, int *groups, double *recompute_ms) {
  if (!h) return HMC_EARG;
  if (windows) *windows = h->c.last_windows;
  if (window_loci) *window_loci = h->c.last_window_loci;
  if (groups) *groups = h->c.last_window_groups;
  if (recompute_ms) *recompute_ms = h->c.ms_ck;
  return HMC_OK;
}

int hmc_last_host_phases(const hmc_ctx *h, double *ms, int n) {
  if (!h || !ms || n <= 0) return HMC_EARG;
  for (int k = 0; k < n && k < hmc::Ctx::HP_N; ++k) ms[k] = h->c.hp_ms[k];
  return hmc::Ctx::HP_N;
}

int hmc_last_estep_restarts(const hmc_ctx *h, int *restarts, double *window_scale) {
  if (!h) return HMC_EARG;
  if (restarts) *restarts = h->c.n_restarts;
  if (window_scale) *window_scale = h->c.win_scale;
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

int hmc_last_mine_reduction(const hmc_ctx *h, double *ms, int *levels) {
  if (!h) return HMC_EARG;
  if (ms) *ms = h->c.ms_red;
  if (levels) *levels = h->c.n_red_levels;
  return HMC_OK;
}

int hmc_set_structure_tier(hmc_ctx *h, int key_mult10, int contrib_mult10) {
  if (!h || key_mult10 < 0 || contrib_mult10 < 0 || key_mult10 > 160 || contrib_mult10 > 160) return HMC_EARG;
  h->c.s1_kmul = key_mult10;
  h->c.s1_cmul = contrib_mult10;
  return HMC_OK;
}

int hmc_set_key_probes(hmc_ctx *h, int probes) {
  if (!h || probes < 1 || probes > 4096) return HMC_EARG;
  h->c.key_probes = probes;
  return HMC_OK;
}

int hmc_comm_stats(const hmc_ctx *h, int64_t *sends, int64_t *recvs, uint64_t *bytes_received) {
  if (!h) return HMC_EARG;
  if (sends) *sends = h->c.p2p_sends;
  if (recvs) *recvs = h->c.p2p_recvs;
  if (bytes_received) *bytes_received = h->c.p2p_bytes;
  return HMC_OK;
}

int hmc_set_comm_timeout(hmc_ctx *h, double seconds) {
  if (!h || !(seconds > 0)) return HMC_EARG;
  h->c.comm_timeout_s = seconds;
  return HMC_OK;
}

int hmc_debug_stall(hmc_ctx *h, double ms) {
  if (!h || !(ms > 0) || ms > 60000) return HMC_EARG;
  hmc::Ctx &c = h->c;
  if (int rc = c.comm_ok()) return rc;
  hipError_t e;
  if ((e = hmc::launch_stall(ms, c.st)) || (e = c.sync_st())) return c.hipfail(e, "debug_stall");
  return HMC_OK;
}

int hmc_model_save(hmc_ctx *h) { return h ? h->c.model_save() : HMC_EARG; }
int hmc_em_rewind(hmc_ctx *h) { return h ? h->c.em_rewind() : HMC_EARG; }

const char *hmc_build_info(void) {
#ifdef HMC_VARIANTS
  return "hmc_amd 0.4+variants gfx950 -O3 -ffp-contract=off, built " __DATE__ " " __TIME__;
#else
  return "hmc_amd 0.4 gfx950 -O3 -ffp-contract=off, built " __DATE__ " " __TIME__;
#endif
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
      (e = c.sync_st()))
    return c.hipfail(e, "get_patterns");
  if (start) memcpy(start, st.data(), (size_t)P * 4);
  if (len) memcpy(len, ln.data(), (size_t)P * 4);
  if (succ) {
    std::vector<uint32_t> s((size_t)P * A);
    if ((e = hipMemcpyAsync(s.data(), c.t_succ.p, s.size() * 4, hipMemcpyDeviceToHost, c.st)) ||
        (e = c.sync_st()))
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
      (e = c.sync_st()))
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
        (e = c.sync_st()))
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
      (e = h->c.sync_st()))
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
      (e = h->c.sync_st()))
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
        (e = c.sync_st()))
      return c.hipfail(e, "get_samples");
    for (int s = 0; s < H; ++s)
      for (int k = 0; k < L; ++k) alleles[(size_t)s * L + k] = c.pan.symbol(k, rows[(size_t)c.h_rowmap[s] * L + k]);
  }
  if (weights && H) {
    if ((e = hipMemcpyAsync(weights, c.d_w.p, (size_t)H * 8, hipMemcpyDeviceToHost, c.st)) ||
        (e = c.sync_st()))
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
