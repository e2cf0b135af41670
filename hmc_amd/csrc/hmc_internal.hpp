// hmc_internal.hpp — device-side data layout shared by the HIP kernels and the
// host runtime of libhmc_amd.  Nothing here crosses the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hmc {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint8_t MISSING = 0xFF;
constexpr int S_MAX = 64;    // sample_size limit (lists of 2S links: segments of one wavefront up to
                             // S = 32, one list per wave over two lanes' slots above; fused kernel: 32)
constexpr int A_MAX = 64;    // alleles per locus limit (allele indices are u8; exact M-step: 44)
constexpr int WAVE = 64;
constexpr int EXACT_C_MAX = (1 << 22) - 1;  // contributions per locus in an exact-M-step record (22-bit field)

// Link metadata word (one k-best entry, HaploPairLink HaploPair.h:14-28):
//   bits 0-15 predecessor state, 16-23 index in the predecessor's list,
//   bit 24 reversed, bit 25 homozygous, bit 26 head (link == NULL).
// State ids (positions in a locus's frontier) take F_BITS bits: frontiers of
// up to F_MAX states per individual and locus.
constexpr int F_BITS = 21;
constexpr uint32_t F_MASK = (1u << F_BITS) - 1u;
constexpr int F_MAX = (int)F_MASK;  // 2 097 151
// Link word (a k-best list entry, also the trace store's): predecessor state,
// index in its list, and the reversed / homozygous / head flags.
__host__ __device__ inline uint32_t meta_pack(uint32_t pred, uint32_t idx, bool rev, bool homo, bool head) {
  return (pred & F_MASK) | ((idx & 0xFFu) << F_BITS) | (rev ? 1u << 29 : 0u) | (homo ? 1u << 30 : 0u) |
         (head ? 1u << 31 : 0u);
}
__host__ __device__ inline uint32_t meta_pred(uint32_t m) { return m & F_MASK; }
__host__ __device__ inline uint32_t meta_idx(uint32_t m) { return (m >> F_BITS) & 0xFFu; }
__host__ __device__ inline bool meta_rev(uint32_t m) { return (m >> 29) & 1u; }
__host__ __device__ inline bool meta_homo(uint32_t m) { return (m >> 30) & 1u; }
__host__ __device__ inline bool meta_head(uint32_t m) { return (m >> 31) & 1u; }
// Contribution word of the structure records: predecessor state, reversed
// flag, and (bits 24..31) the predecessor's list length.
constexpr uint32_t CW_REV = 1u << F_BITS;
__host__ __device__ inline uint32_t cw_pack(uint32_t s, bool rev) { return s | (rev ? CW_REV : 0u); }
__host__ __device__ inline uint32_t cw_state(uint32_t w) { return w & F_MASK; }
__host__ __device__ inline bool cw_rev(uint32_t w) { return (w >> F_BITS) & 1u; }
__host__ __device__ inline uint32_t cw_ns(uint32_t w) { return w >> 24; }
// Exact-mode forward-link words (the records' extendAll list) carry in bits
// 22..31 the target state's unordered allele pair max(a,b)(max(a,b)+1)/2 +
// min(a,b) (< 990: at most 44 alleles per locus in exact mode), so the trie
// walk tests a target's alleles without reading its header.
constexpr int XPAIR_SHIFT = F_BITS + 1;
__host__ __device__ inline uint32_t xpair_index(uint32_t a, uint32_t b) {
  const uint32_t x = a > b ? a : b, y = a > b ? b : a;
  return x * (x + 1) / 2 + y;
}
__host__ __device__ inline uint32_t cw_xpair(uint32_t w) { return w >> XPAIR_SHIFT; }

// Per-state trace header word: last allele of pattern a / b, link count.
__host__ __device__ inline uint32_t hdr_pack(uint32_t al_a, uint32_t al_b, uint32_t n) {
  return (al_a & 0xFFu) | ((al_b & 0xFFu) << 8) | ((n & 0xFFu) << 16);
}

// Structure-record header word of a state (estep_split.hip): bit 27 marks a
// state whose adds overflow S (a chain of selections in the value pass).
constexpr uint32_t HDR_CHAIN = 1u << 27;

// E-step status codes written per individual.
enum EStatus : int32_t {
  EST_OK = 0,
  EST_UNRESOLVED = 1,          // dead frontier (HaploBuilder.cpp:80-81)
  EST_OVERFLOW_FRONTIER = -1,  // more states than the per-wave capacity
  EST_OVERFLOW_TRACE = -2,     // trace buffer exhausted
  EST_NO_HEAD_PATTERN = -3,    // "Can not find matching pattern!" (HaploBuilder.cpp:215-217)
  EST_OVERFLOW_REC = -4,       // structure-record store exhausted (split E-step)
  EST_OVERFLOW_CONTRIB = -5,   // more contributions at a locus than the structure pass's capacity
  EST_DF_STALL = -6,           // dataflow value pass: a wait made no progress (watchdog; a bug, reported)
  EST_OVERFLOW_CKPT = -7,      // windowed E-step: the checkpoint store is full
  EST_OVERFLOW_NODES = -8,     // windowed E-step: the trace-survivor node store is full
  EST_GC_MISS = -9,            // windowed E-step: a survivor's predecessor is not in the boundary list (a bug)
  EST_NEEDS_EXACT = 2,         // split E-step: a forward likelihood underflowed to 0 before
                               // the last locus, so extend() would skip that pair
                               // (HaploBuilder.cpp:237) — re-run on the fused kernel
  EST_NEEDS_ORDER = 3,         // value-only value pass: a tie makes the result depend on
                               // the libstdc++ list order — re-run on the exact value pass
  EST_OK_PRUNED = 4,           // structure records built with extend()'s forward test
                               // (HaploBuilder.cpp:237): pairs whose forward likelihood is 0
                               // are not extended; the value pass then expects zeros
};

// Panel resident in HBM.
struct DevPanel {
  int N = 0, L = 0, amax = 0;
  uchar2 *geno_im = nullptr;   // [N][L] (allele index of haplotype 0, 1), 0xFF missing
  uchar2 *geno_lm = nullptr;   // [L][N] same, locus-major (genotype-branch mining)
  uint8_t *anum = nullptr;     // [L]
  double *afreq = nullptr;     // [L][amax]
};

// Pattern model resident in HBM (PatternManager after initialize()).
struct DevModel {
  int P = 0;
  uint32_t *succ = nullptr;    // [P][amax]
  double *tp = nullptr;        // [P]
  double *freq = nullptr;      // [P]
  uint8_t *last = nullptr;     // [P] last allele index
  int n_head = 0, head_len = 1;
  uint32_t *head_ids = nullptr;   // [n_head], id order
  uint32_t *head_pat0 = nullptr;  // [amax+1] pattern id of (locus 0, allele x); [amax] = missing allele
  // head_len > 1: initHeadList's head pairs per individual, computed on the
  // host (HaploBuilder.cpp:153-224), indexed by global individual - hf_base
  int hf_base = 0;
  const uint32_t *hf_off = nullptr;    // [n+1]
  const uint32_t *hf_pairs = nullptr;  // [2 x total] (head id, matching pattern id)
  const int32_t *hf_status = nullptr;  // [n] EST_OK or EST_NO_HEAD_PATTERN
  const uint8_t *head_al = nullptr;    // [P][head_len] alleles of the start-0 length-head_len patterns
  // the same table in end-locus order (gmodel.hip), when built: g = position
  // of a pattern among those sorted by (end locus, id); the structure pass
  // (estep_structure) then carries g instead of ids
  const uint32_t *gsucc = nullptr;  // [P][amax] g of the successor, NONE
  const double *gtp = nullptr;      // [P] by g
  const uint8_t *glast = nullptr;   // [P] by g
  const uint32_t *gid = nullptr;    // [P] g -> id
  const uint32_t *ginv = nullptr;   // [P] id -> g
};

// Build of the end-locus-ordered table (gmodel.hip): sort temporaries and outputs.
struct GModelArgs {
  int P = 0, A = 0, L = 0;
  const int32_t *start = nullptr, *len = nullptr;
  const uint32_t *succ = nullptr;
  const double *tp = nullptr;
  const uint8_t *last = nullptr;
  uint32_t *key_in = nullptr, *key_out = nullptr, *id_in = nullptr;  // [P] each
  void *temp = nullptr;
  size_t temp_bytes = 0;
  uint32_t *gid = nullptr, *inv = nullptr, *gsucc = nullptr;
  double *gtp = nullptr;
  uint8_t *glast = nullptr;
};
size_t gmodel_sort_bytes(int P, int L);
hipError_t build_gmodel(const GModelArgs &g, hipStream_t st);

struct EstepArgs {
  DevPanel pan;
  DevModel mod;
  int S;
  int indiv_begin, indiv_end;  // batch [begin, end)
  // per-wave scratch
  char *scratch;
  size_t scratch_stride;
  int fcap, hcap;    // HBM tier capacities (states, key slots)
  int lds_fc, lds_hc;  // LDS tier: states per frontier, key slots (power of two)
  // trace store
  uint32_t *trace;
  unsigned long long trace_cap;     // words
  unsigned long long *trace_cursor; // bump allocator (when trace_base is null)
  const unsigned long long *trace_base;  // [batch] reserved trace region of each individual, or null
  unsigned long long *loc_off;      // [batch][L+1] word offsets
  // per-individual outputs (indexed by individual - indiv_begin)
  double *total;
  int32_t *ncand;
  int32_t *status;
  uint32_t *cand_state;  // [batch][S_MAX]
  uint32_t *cand_idx;    // [batch][S_MAX]
  double *prior;         // [batch][S_MAX]
  double *posterior;     // [batch][S_MAX]
  double *weight;        // [batch][S_MAX]
  unsigned long long *re_count;  // [batch]
  unsigned int *max_states;      // [1] running maximum frontier size
  int32_t *fmax;                 // [batch] largest frontier of each individual
  const int32_t *order;          // [batch] individuals in block-visit order (nullptr: natural order)
  int n_order;                   // entries of `order` to visit (the whole batch unless re-running a subset)
  int32_t *cost;                 // [batch] shader kcycles spent per individual (scheduling hint)
  unsigned long long *stamps;    // [20] diagnostic build: shader cycles per phase
  int diag_indiv;                // diagnostic build: stamp only this batch index (-1: all)
};

// Locus window of the checkpoint-and-recompute E-step (see StructArgs).
// Checkpoint of an individual's frontier after record index j (window start
// j + 1), at word ck_off[b * (nwin + 1) + win] of ck_in / ck_out (even):
//   [F][0] | lo u32[F] hi u32[F] nl u32[F] (structure: pattern g / ids and list
//   lengths) | pad to even | fwd f64[F] hm u64[F] lik f64[F][S] (value pass)
struct WinArgs {
  int lo = 0, hi = 0;             // record / trace indices [lo, hi); hi == L + 1: the last window
  int win = 0, nwin = 1;
  const uint32_t *ck_in = nullptr;  // the checkpoints this window starts from (offsets ck_off[b][win])
  uint32_t *ck_out = nullptr;       // the checkpoints it leaves (offsets ck_off[b][win + 1])
  unsigned long long ck_cap = 0;  // words of ck_out
  unsigned long long *ck_cursor = nullptr;  // next free word of ck_out
  unsigned long long *ck_off = nullptr;  // [batch][nwin + 1]
  bool ck_write = false;          // save the window's last frontier (forward passes)
  __host__ __device__ bool windowed() const { return ck_out != nullptr; }
};
__host__ __device__ inline unsigned long long ck_value_off(unsigned long long F) { return (2ull + 3ull * F + 1ull) & ~1ull; }
__host__ __device__ inline unsigned long long ck_words(unsigned long long F, int S) {
  return ck_value_off(F) + 4ull * F + 2ull * F * (unsigned long long)S;
}

// Split E-step, pass 1 (estep_structure): the value-independent part of
// resolve() — frontier pattern-id pairs, successor keys, m_best_pair dedup in
// creation order, per-state contribution lists and k-best list lengths — as
// per-locus structure records.  Pass 2 (estep_values) replays them with the
// likelihood arithmetic.  Record of locus j at word rec_off[b][j] (even):
//   [F][C][NCH][0] tpv f64[F] | hdr u32[F] (last allele a | b<<8 | nl<<16 |
//   homo<<24 at the head) | cbeg u32[F+1] | contrib u32[C] (pred state |
//   reversed<<16 | pred list length<<24), each state's in add order |
//   chains u32[NCH] (states whose adds overflow S, most contributions first).
struct StructArgs {
  DevPanel pan;
  DevModel mod;
  int S;
  int indiv_begin;
  const int32_t *order;
  int n_order;
  char *scratch;
  size_t scratch_stride;
  int fcap, hcap, ccap;           // HBM tier capacities: states, key slots, contributions per locus
  int lds_fc, lds_hc, lds_cc;     // LDS tier
  uint32_t *rec;
  unsigned long long rec_cap;     // words
  unsigned long long *rec_cursor; // bump allocator (when rec_base is null)
  const unsigned long long *rec_base;  // [batch] reserved record region of each individual, or null
  const unsigned long long *rec_size;  // [batch] its size in words (null: unbounded, the exact need)
  unsigned long long *rec_off;    // [batch][L+1]
  // Exact store needs of each individual (words): its records and its value-pass
  // trace.  An individual whose records do not fit the store keeps walking the
  // loci without writing them (status EST_OVERFLOW_REC) so both are known.
  unsigned long long *rec_need;   // [batch]
  unsigned long long *trace_need; // [batch]
  // Exact M-step (--exact-estimate): the records also carry the head pairs'
  // pattern ids, each locus's contributions in extendAll order (target state |
  // reversed<<16, NONE when a successor is missing) and its allele pairs'
  // orientation counts — the forward links of HaploPair (HaploPair.cpp:44,67)
  // in push order; trace_need then counts the fwd/bwd store (4 words/state).
  bool exact;
  // extend()'s test (HaploBuilder.cpp:237): forward likelihoods are summed per
  // state as the records are built and a pair whose sum is 0 is not extended.
  // For individuals whose likelihoods underflow (the value pass reports
  // EST_NEEDS_EXACT); status EST_OK_PRUNED.  Scratch: estep_s1_scratch_bytes(.., prune)
  bool prune = false;
  int probe_lds = 16;  // LDS probes of the key table before the HBM table (PROBE_LDS)
  int32_t *next_q;                // dynamic schedule: order entries taken after the first gridDim.x (zeroed)
  // Locus windows (checkpoint-and-recompute E-step, Ctx::estep_windowed):
  // records of indices [win_lo, win_hi) only — win_lo == head_len starts
  // with the head pairs, else from the frontier the checkpoint of window
  // `win` holds (ck_off[b][win]); a window that ends before L+1 saves its
  // last frontier as window win+1's checkpoint when ck_write (allocating it
  // from ck_cursor).  Classic passes: win_lo = head_len, win_hi = L + 1.
  WinArgs w;
  int32_t *status;                // [batch]
  unsigned long long *re_count;   // [batch] (re_mode: 0 written, 1 added to, 2 untouched)
  int re_mode = 0;
  int32_t *fmax;                  // [batch]
  unsigned int *max_states;
  unsigned long long *stamps;     // diagnostic build: [16] shader cycles per phase / counters
};

// Trace words one locus with F states takes (header, F header words, pad, F x S
// link words; the layout of trace_links()).
__host__ __device__ inline unsigned long long trace_locus_words(unsigned long long F, int S) {
  return 2ull + F * (1ull + (unsigned long long)S);
}

struct ValueArgs {
  int S, L, head_len;
  const int32_t *order;
  int n_order;
  const uint32_t *rec;
  const unsigned long long *rec_off;
  char *scratch;
  size_t scratch_stride;
  int fcap, lds_fc;
  int32_t *next_q;  // dynamic schedule: order entries taken after the first gridDim.x (zeroed)
  uint32_t *trace;
  unsigned long long trace_cap;
  unsigned long long *trace_cursor;
  const unsigned long long *trace_base;  // [batch] reserved trace region of each individual, or null
  unsigned long long *loc_off;
  int32_t *status;  // in: pass-1 status; out: EST_OK / EST_NEEDS_EXACT / EST_OVERFLOW_TRACE
  double *total;
  int32_t *ncand;
  uint32_t *cand_state, *cand_idx;
  double *prior, *posterior, *weight;
  int32_t *cost;
  unsigned long long *stamps;  // diagnostic build: [16] block-critical-path cycles per phase
  WinArgs w;                   // locus window (StructArgs::w); cost is added to over the forward windows
};

struct TracebackArgs {
  int L, S, head_len, nbatch;      // nbatch: entries of `order` (or individuals 0..nbatch-1 when null)
  const int32_t *order;
  int indiv_begin;                 // global index of the batch's first individual
  DevModel mod;                    // head pairs / alleles when head_len > 1
  const uint32_t *trace;
  const unsigned long long *loc_off;
  const int32_t *ncand;
  const uint32_t *cand_state, *cand_idx;
  const double *weight;
  const int32_t *sample_base;  // [batch] first sample row of each individual
  uint8_t *rows;               // [H][L] sample-major haplotypes (allele index)
  double *w_out;               // [H]
  // Windowed E-step (trace garbage collection, TraceGcArgs): trace indices
  // below full_lo are no longer in the trace store; the walk continues at
  // index full_lo - 1 in the survivor nodes — the entry (state, list index)
  // found by key in the individual's boundary list, then the nodes' chain.
  // full_lo = 0: every trace index is in the store.
  int full_lo = 0;
  const uint32_t *nodes = nullptr;                // 3 words per node: key, alleles | rev << 16, predecessor node
  const unsigned long long *bnd_off = nullptr;    // [batch] first node of the boundary list
  const uint32_t *bnd_n = nullptr;                // [batch] its length
};

// Trace garbage collection of the windowed E-step (estep_trace_gc): the
// k-best traces of loci [lo0, mid) (the older of two windows whose full traces
// are in the store) shrink to their survivors — the list entries reachable
// backward from any entry at the last locus of [mid, hi1).  Survivors become
// nodes (key = state << 8 | list index, the pair's last alleles and the link's
// reversed flag, the predecessor's node), locus by locus in key order; the
// last locus's nodes are the individual's boundary list, through which the
// next window's survivors and the final traceback find their predecessors.
struct TraceGcArgs {
  int L = 0, S = 1, head_len = 1;
  const int32_t *order = nullptr;
  int n_order = 0;
  int32_t *next_q = nullptr;
  const uint32_t *trace = nullptr;
  const unsigned long long *loc_off = nullptr;
  int lo0 = 0, mid = 0, hi1 = 0;
  uint32_t *scratch = nullptr;  // per block: mark offsets, two prefix rows, the reached-entry bitmaps
  size_t scratch_stride = 0;    // words
  int max_words = 1;            // bitmap words of the largest locus (F x S bits)
  uint32_t *nodes = nullptr;
  unsigned long long node_cap = 0;       // nodes
  unsigned long long *node_cursor = nullptr;
  unsigned long long *bnd_off = nullptr;  // [batch]
  uint32_t *bnd_n = nullptr;              // [batch]
  int32_t *status = nullptr;              // EST_OVERFLOW_NODES: the node store is full (nothing changed)
};
hipError_t launch_estep_trace_gc(const TraceGcArgs &a, int grid, hipStream_t st, int nw = 1);

size_t estep_scratch_bytes(int fcap, int hcap, int S, int nw);
size_t estep_lds_bytes(int S, int fc, int hc, int nw, int amax);
hipError_t launch_test_coop_nth(double *lik, uint32_t *tag, const int *off, const int *n, const int *nth, int count, int sw, hipStream_t st);
hipError_t launch_estep(const EstepArgs &a, int grid, int nw, hipStream_t st);
size_t estep_s1_scratch_bytes(int fcap, int hcap, int ccap, int nw, bool prune = false);
size_t estep_s1_lds_bytes(int fc, int hc, int cc, int amax, int nw);
size_t estep_s2_scratch_bytes(int fcap, int S);
size_t estep_s2_lds_bytes(int S, int fc, int nw, bool pair = false);
// nw: wavefronts per individual, 1 or 4
hipError_t launch_estep_structure(const StructArgs &a, int grid, int nw, hipStream_t st);
// The same records with fewer block hand-offs per locus (estep_split.hip,
// "pass 1, v2"); sized with estep_s1v2_lds_bytes and estep_s1_scratch_bytes(.., nw = 2, ..).
size_t estep_s1v2_lds_bytes(int fc, int hc, int cc, int amax, int nw);
hipError_t launch_estep_structure2(const StructArgs &a, int grid, int nw, hipStream_t st);
// wpe: 4 or 5 resident waves per SIMD (register budget of the instantiation)
hipError_t launch_estep_values(const ValueArgs &a, int grid, int nw, bool fast, int wpe, hipStream_t st,
                               bool pair = false);
// Dataflow value pass (estep_df.hip): one A wave + nw-1 B waves per
// individual, a ring of R >= 3 frontiers, a chain queue of qcap (power of two)
// slots.  S <= 32 (pair: S <= 16), exact order only, trace_base required.
size_t estep_df_lds_bytes(int S, int fc, int nw, int na, bool pair, int R, int qcap, int fcap);
size_t estep_df_scratch_bytes(int fcap, int S, int R);
hipError_t launch_estep_values_df(const ValueArgs &a, int grid, int nw, int na, int wpe, bool pair, int R, int qcap,
                                  hipStream_t st);
hipError_t launch_traceback(const TracebackArgs &a, int total_cands, hipStream_t st);
hipError_t launch_transpose_rows_u8(const uint8_t *in, const int32_t *rowmap, uint8_t *out, int rows, int cols,
                                    hipStream_t st);
hipError_t launch_transpose_u8(const uint8_t *in, uint8_t *out, int rows, int cols, int ld_out, int col0,
                               hipStream_t st);
hipError_t launch_gather_resolutions(const uint8_t *rows, int L, const int32_t *sbase, const int32_t *ncand,
                                     const uchar2 *geno_im, int i0, int n, uint8_t *out, hipStream_t st);
hipError_t launch_haplocomp_counts(const uchar2 *geno_im, int i0, int n, int L, const uint8_t *res, int32_t *cnt,
                                   int32_t *bad, hipStream_t st);
hipError_t launch_stall(double ms, hipStream_t st);  // hmc_debug_stall (mstep.hip)
hipError_t launch_scan_i32(const int32_t *in, int32_t *out_excl, int n, int mul, int32_t *total, hipStream_t st);

}  // namespace hmc
