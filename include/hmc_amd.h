/* hmc_amd.h — C-ABI of libhmc_amd.so, the MI355X-native HaploModel EM.
 *
 * The reference (Wu-Lab/HMC v0.9.1) has no plugin or FFI surface: its hot path
 * is the C++ class seam HaploModel::run -> HaploBuilder::resolve /
 * PatternManager::findPatternByFreq inside one binary.  Each entry point below
 * replaces one of those seams; the citation names the reference interface it
 * stands in for.  Conventions:
 *   - plain pointers and sizes, no C++ or torch types;
 *   - host buffers are caller-owned, device buffers are owned by the context;
 *   - every function returns 0 (HMC_OK) or a negative HMC_E* code; the text of
 *     the last failure is available from hmc_ctx_error().  The reference's
 *     fatal errors (Logger::error + exit(1)) become return codes here;
 *   - allele symbols are the reference's Allele values (the ASCII code for SNP
 *     'S' loci, the integer for microsatellite 'M' loci), -1 = missing;
 *   - one host thread per context.
 */
#ifndef HMC_AMD_H
#define HMC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HMC_OK 0
#define HMC_EARG -1         /* invalid argument / call order */
#define HMC_EHIP -2         /* HIP runtime failure */
#define HMC_EIO -3          /* file could not be read or written */
#define HMC_EUNSUPPORTED -4 /* parameter outside what the GPU path implements */
#define HMC_ENOPATTERN -5   /* "Can not find matching pattern!" (HaploBuilder.cpp:215-217) */
#define HMC_ERCCL -6        /* RCCL failure */
#define HMC_ENOMEM -7       /* device memory exhausted */

typedef struct hmc_ctx hmc_ctx;

/* ---- context ---------------------------------------------------------- */
/* One context per GPU.  Replaces constructing HaploModel (HaploModel.h:29). */
int hmc_ctx_create(int device, hmc_ctx **out);
/* Multi-GPU: one process per GPU; `unique_id` = 128 bytes from
 * hmc_rccl_unique_id() on rank 0, broadcast by the caller.  Individuals are
 * sharded in contiguous blocks; the M-step all-reduces per-level sums. */
int hmc_rccl_unique_id(void *out128);
int hmc_ctx_create_dist(int device, int rank, int world, const void *unique_id, hmc_ctx **out);
/* Multi-GPU on a communicator the caller already owns (an ncclComm_t, RCCL):
 * rank and world are taken from it; hmc_ctx_destroy leaves it alive.  The
 * seam of SURVEY.md §8(b) (hmc_ctx_create(device, rccl_comm_or_null, ...)),
 * replacing HaploModel's construction (HaploModel.h:29) inside a host that
 * runs its own RCCL. */
int hmc_ctx_create_comm(int device, void *rccl_comm, hmc_ctx **out);
/* An RCCL communicator made by the RCCL this library is linked with (for
 * hosts without their own RCCL binding, and tests: a communicator from a
 * second copy of librccl in the process would not be usable here). */
int hmc_rccl_comm_init(int device, int world, int rank, const void *unique_id, void **comm);
int hmc_rccl_comm_destroy(void *comm);
/* Same sharding with a caller-supplied collective instead of RCCL: fn must
 * sum `n` doubles element-wise across ranks in place and return 0.  Lets
 * several ranks share one GPU (tests) or run over any host transport. */
typedef int (*hmc_allreduce_fn)(double *buf, size_t n, void *user);
int hmc_ctx_create_hostcoll(int device, int rank, int world, hmc_allreduce_fn fn, void *user, hmc_ctx **out);
/* Test hook: a one-rank context made with a unique id or a communicator runs
 * every collective of the sharded path anyway (results unchanged), so the
 * RCCL calls are exercised on a one-GPU machine.  HMC_EARG on a context
 * without a communicator. */
int hmc_set_force_collectives(hmc_ctx *ctx, int on);
void hmc_ctx_destroy(hmc_ctx *ctx);
const char *hmc_ctx_error(const hmc_ctx *ctx);

/* Cross-rank sums of a sharded run (M-step candidate sums per mining level,
 * log-likelihood, total sample weight).  0 (default) = ordered: rank r
 * continues each running sum of ranks 0..r-1 over its contiguous block of
 * items, which reproduces the reference's sequential sums
 * (PatternManager.cpp:254-262, HaploModel.cpp:110, HaploData.cpp:120-126) bit
 * for bit — a point-to-point chain per mining level (ncclRecv from r-1,
 * the rank's adds, ncclSend to r+1; one ncclBroadcast from W-1); 1 = all-reduce of per-rank
 * partial sums (one collective, sums reassociated: last-bit drift, which can
 * flip a pattern at the min_freq threshold). */
int hmc_set_reduction(hmc_ctx *ctx, int mode);

/* HaploModel public parameters (HaploModel.h:15-26; CLI defaults HMC.cpp:35-47).
 * min_freq_abs > 0 overrides min_freq exactly as HaploModel::findPatterns does
 * (HaploModel.cpp:54-56).  sample_size 1..64 (HaploPair's k-best lists,
 * HaploBuilder.cpp:44, HaploPair.cpp:85-88; above 32 the split E-step only);
 * larger values fail the E-step with HMC_EUNSUPPORTED. */
int hmc_set_params(hmc_ctx *ctx, double min_freq_abs, double min_freq, int min_pattern_len, int max_pattern_len,
                   int sample_size);

/* HaploModel::setModel + mc_order (HaploModel.cpp:26-36, 65-76; HMC.cpp:35,41):
 * "MV" (default; patterns by frequency), "MC" (Markov chain of order mc_order:
 * PatternManager::findPatternBlock(mc_order+1), every candidate of that length,
 * head length mc_order+1), "MA" (MV; its adjustFrequency only range-checks). */
int hmc_set_model(hmc_ctx *ctx, const char *model, int mc_order);
/* HaploModel::exact_estimate (--exact-estimate, HMC.cpp:42; HaploModel.cpp:
 * 140-141): after an E-step, hmc_find_patterns (and hmc_run) re-estimate the
 * table with PatternManager::estimatePatterns (PatternManager.cpp:364-438):
 * expected pattern counts under the current model, from a forward-backward
 * pass and a ForwardPatternTree walk per individual and start locus
 * (HaploBuilder.cpp:263-450), candidates grown by extendPatterns; M0 still
 * mines the genotypes.  Model MC re-estimates the table in place.
 * Frequencies agree with the reference to rounding (its sums run in pointer
 * order); they are deterministic and independent of the sharding. */
int hmc_set_exact_estimate(hmc_ctx *ctx, int on);
/* Last exact M-step: rounds of estimateFrequency, candidates estimated, and
 * device ms of the trie walks. */
int hmc_last_exact_stats(const hmc_ctx *ctx, int *rounds, uint64_t *candidates, double *walk_ms);
/* The last exact M-step's breadth-first walk: work units (trie nodes of an
 * individual and start locus), kernel launches, units deferred for room, and
 * the individuals walked over pruned records (forward likelihoods that
 * underflow: extend()'s test, HaploBuilder.cpp:237, 291-314). */
int hmc_last_exact_walk(const hmc_ctx *ctx, int64_t *units, int64_t *launches, int64_t *deferred, int *pruned);
/* HaploModel::num_patterns (HMC.cpp:38): > 0 mines with
 * PatternManager::findPatternByNum (PatternManager.cpp:44-70, models MV/MA);
 * <= 0 (default) with findPatternByFreq. */
int hmc_set_num_patterns(hmc_ctx *ctx, int num_patterns);

/* ---- panel (GenoData / HaploFile) --------------------------------------- */
/* HaploFile::readGenoData for the PHASE format (HaploFile.cpp:54-118). */
int hmc_load_phase(hmc_ctx *ctx, const char *path);
/* Same panel from memory: alleles[N][2][L] symbols, types[L] ('S' or 'M').
 * Runs GenoData::checkAlleleSymbol (GenoData.cpp:78-118) and uploads. */
int hmc_load_genotypes(hmc_ctx *ctx, int N, int L, const int32_t *alleles, const char *types);
int hmc_panel_info(const hmc_ctx *ctx, int *N, int *L, int *max_alleles);
/* This rank's individuals [i0, i1): contiguous blocks balanced by E-step cost
 * (L/8 + heterozygous-or-missing loci per individual); [0, N) on one rank. */
int hmc_shard_range(const hmc_ctx *ctx, int *i0, int *i1);
/* Measurement hook of a one-rank context: from here on the E-step and the
 * M-step's scans cover individuals [i0, i1) of the loaded panel only, with
 * the current model (e.g. the M0 mined over the whole panel) — rank r's own
 * E-step work of an N-rank run, on one GPU (tools/cfg4_rank.py).  Drops the
 * samples and every per-individual estimate.  Replaces no reference
 * interface. */
int hmc_set_shard(hmc_ctx *ctx, int i0, int i1);
/* Per-locus allele tables: num[L], sym[L][max_alleles], freq[L][max_alleles]
 * (GenoData::allele_num / allele_symbol / allele_frequency, GenoData.h:43-49). */
int hmc_allele_table(const hmc_ctx *ctx, int32_t *num, int32_t *sym, double *freq);

/* ---- M-step: PatternManager::findPatternByFreq (PatternManager.cpp:27-42) --
 * Mines from the genotypes while no E-step samples exist (M0), from the
 * weighted samples afterwards, then runs initialize() (ids, head list,
 * successors).  *n_patterns = patterns found; *r_m = candidate x item scan
 * steps (SURVEY.md §8d R_M, local to this rank). */
int hmc_find_patterns(hmc_ctx *ctx, int *n_patterns, uint64_t *r_m);
/* Per-level seam of the same search: PatternManager::checkFrequency
 * (PatternManager.cpp:146-193, called for each candidate by searchPattern
 * :100-144) for n caller-given candidates of length `level` — start[n],
 * alleles[n][level] as symbols.  freq[c] = the pattern frequency the reference
 * assigns: genotype branch (no samples yet) sum over individuals of
 * getMatchingFrequency (:267-291) / N, sample branch sum of matching sample
 * weights / total weight; sums in item order and, across ranks, in rank order
 * (hmc_set_reduction).  *scanned = n x items of this rank. */
int hmc_mine_level(hmc_ctx *ctx, int level, int n, const int32_t *start, const int32_t *alleles, double *freq,
                   uint64_t *scanned);
int hmc_model_info(const hmc_ctx *ctx, int *n_patterns, int *head_len);
/* Blocks of start loci for the search (0 = automatic: one block up to about
 * 2.5e7 individual-loci of panel, else blocks of about that size; always one
 * block for findPatternByNum and heads longer than 1 locus).  The roots of
 * searchPattern's DFS are independent (PatternManager.cpp:90-108): blocks
 * from locus L-1 down give the same table, ids and successors, with the
 * candidate-node memory of two blocks and the matching lists of one, for any
 * pattern length.  A block whose nodes or lists do not fit in device memory
 * (or in hmc_set_mine_memory's cap) is re-run with half the width, and the
 * blocks below it keep that width. */
int hmc_set_mine_block(hmc_ctx *ctx, int start_loci);
/* Last E-step: the largest frontier (states at one locus of one individual)
 * and the state capacity it ran with (grows by doubling on overflow, up to
 * 2 097 151 states: 21-bit state ids in the records and list links). */
int hmc_last_estep_frontier(hmc_ctx *ctx, int *max_states, int *frontier_cap);
/* Cap on one search level's matching lists, in bytes (0 = device memory
 * only; 12 B per entry of the genotype branch, 4 B of the sample branch):
 * a level over the cap splits its block as if memory had run out. */
int hmc_set_mine_memory(hmc_ctx *ctx, uint64_t list_bytes);
/* Last search: blocks, candidate nodes created (all blocks) and the size of
 * the node arrays kept (GB, ~70 B per node). */
int hmc_last_mine_stats(const hmc_ctx *ctx, int *blocks, int64_t *nodes, double *node_window_gb);
/* Cross-rank reduction of the last pattern search (multi-rank contexts):
 * device ms from the first to the last collective of each mining level,
 * summed (the ordered chain's mine_sum launches included), and the number of
 * levels reduced.  0 / 0 on one rank.  Replaces no reference interface
 * (the reference is single-process). */
int hmc_last_mine_reduction(const hmc_ctx *ctx, double *ms, int *levels);
/* Point-to-point hops of the ordered chain issued by this context since its
 * creation: ncclSend calls, ncclRecv calls and bytes received (a forced
 * one-rank context sends each hop to itself, grouped).  Replaces no reference
 * interface. */
int hmc_comm_stats(const hmc_ctx *ctx, int64_t *sends, int64_t *recvs, uint64_t *bytes_received);
/* Structure pass (tuning, results unchanged): LDS probes of the key table
 * (m_best_pair) before a key goes to its HBM tier; default 16. */
int hmc_set_key_probes(hmc_ctx *ctx, int probes);
/* Structure pass (tuning, results unchanged): the block's LDS split — key
 * slots and contributions per frontier state, in tenths (0 = defaults: 40 and
 * 20 at 4 waves per individual, 20 and 20 otherwise). */
int hmc_set_structure_tier(hmc_ctx *ctx, int key_mult10, int contrib_mult10);
/* Bounded waits of an RCCL context (default 1800 s): every stream sync polls
 * ncclCommGetAsyncError; on an asynchronous error or after `seconds` without
 * the stream draining, the communicator is aborted (ncclCommAbort — a
 * caller-owned communicator too: do not destroy it afterwards) and the call
 * returns HMC_ERCCL, as does every later collective of the context.  A rank
 * whose neighbour died therefore ends instead of hanging in ncclRecv. */
int hmc_set_comm_timeout(hmc_ctx *ctx, double seconds);
/* Test hook of the bounded wait: keeps the context stream busy for `ms`
 * (one wavefront, bounded) and syncs it through the same wait. */
int hmc_debug_stall(hmc_ctx *ctx, double ms);
/* Pattern table in id order (HaploPattern.h:16-98).  succ[P][max_alleles]
 * holds pattern ids (-1 = none); alleles[P][maxlen] symbols (-1 padding).
 * Any output pointer may be NULL. */
int hmc_get_patterns(hmc_ctx *ctx, int32_t *start, int32_t *len, double *freq, double *prefix, double *tp,
                     int32_t *succ, int32_t *alleles, int maxlen);
/* Install an externally built pattern table (test seam: lets the E-step be
 * checked against another implementation's M-step output).  last_symbol[P] is
 * the pattern's last allele; succ as above. */
int hmc_set_patterns(hmc_ctx *ctx, int P, const int32_t *start, const int32_t *len, const double *freq,
                     const double *tp, const int32_t *succ, const int32_t *last_symbol);

/* ---- E-step: HaploModel::resolveAll (HaploModel.cpp:79-115) ------------
 * Resolves every individual of this rank's shard with HaploBuilder::resolve
 * (HaploBuilder.cpp:35-126), keeps the weighted samples on the device for the
 * next M-step, and returns the log-likelihood (all ranks), the number of
 * samples (this rank) and R_E (retained k-best links, this rank). */
int hmc_resolve_all(hmc_ctx *ctx, double *log_likelihood, int *n_samples, uint64_t *r_e);
/* Per individual of the shard: genotype probability (total forward
 * likelihood), number of candidates, status (0 ok, 1 unresolved), and per
 * candidate [n][sample_size] prior / posterior / sample weight. */
int hmc_get_estep(hmc_ctx *ctx, double *total, int32_t *ncand, int32_t *status, double *prior, double *posterior,
                  double *weight);
/* Largest number of HaploPair states any locus of each individual held in the
 * last E-step (diagnostic). */
int hmc_get_estep_stats(hmc_ctx *ctx, int32_t *fmax);
/* Per individual of the shard: E-step time of the last E-step in units of
 * 1024 shader clocks (value pass; the scheduling key of the next E-step). */
int hmc_get_estep_cost(hmc_ctx *ctx, int32_t *cost);
/* Diagnostic build (libhmc_amd_diag.so) only: shader-cycle / event counters
 * of the last E-step summed over waves, out40[0, 20) the value pass (or fused
 * kernel), out40[20, 36) the structure pass; zeros in the product build. */
int hmc_get_stamps(hmc_ctx *ctx, uint64_t *out40);
/* HaploData samples of this rank: alleles[H][L] symbols, weights[H]. */
int hmc_get_samples(hmc_ctx *ctx, int32_t *alleles, double *weights, double *total_weight);
/* Drop the samples so the next hmc_find_patterns mines the genotypes again
 * (HaploBuilder::setGenoData clears m_samples, HaploBuilder.cpp:19-23). */
int hmc_clear_samples(hmc_ctx *ctx);
/* Selected pair per individual of the last E-step ([n][2][L] symbols;
 * unresolved individuals keep the input genotype, HaploBuilder.cpp:117-124). */
int hmc_get_resolutions(hmc_ctx *ctx, int32_t *out);

/* ---- whole EM: HaploModel::run (HaploModel.cpp:117-155) ------------------ */
typedef struct hmc_iter_log {
  double log_likelihood;
  double t_estep_s, t_mstep_s; /* wall time of E_k and of M_k (0 if no M-step) */
  uint64_t r_e, r_m;
  int n_patterns;              /* patterns after M_k */
  int n_samples;
  /* HaploComp of the input panel (phase as given) against the accepted
   * resolutions after E_k (HaploModel.cpp:134-136) */
  double switch_error, ihp, igp;
} hmc_iter_log;
/* Runs M0 + up to max_iteration EM iterations with the reference's
 * convergence rule.  log[] receives up to log_cap iterations; *iterations the
 * number run; *t_m0_s, *r_m0, *n_patterns0 describe M0. */
int hmc_run(hmc_ctx *ctx, int max_iteration, hmc_iter_log *log, int log_cap, int *iterations, double *t_m0_s,
            uint64_t *r_m0, int *n_patterns0);
/* One iteration of that loop (HaploModel.cpp:130-144) for a host that drives
 * the EM itself, after a first hmc_find_patterns: E-step, accept the
 * resolutions if the LL did not drop below *old_ll, HaploComp, the continue
 * rule (*go), and the M-step when continuing — or always, with always_mstep
 * (a fixed number of steps, as bench.py times).  *old_ll (start: -DBL_MAX)
 * becomes the LL when the M-step ran. */
int hmc_em_iteration(hmc_ctx *ctx, int iteration, int max_iteration, int always_mstep, double *old_ll,
                     hmc_iter_log *log, int *go);
/* Model snapshot for hosts that repeat the EM from one M-step (bench.py runs
 * the reference's converged chain from M0 again and again).  hmc_model_save
 * keeps a device copy of the current pattern table; hmc_em_rewind restores it
 * and returns the EM to the state HaploModel::run has right after build()
 * (HaploModel.cpp:121-129): no samples, resolutions = the input genotypes,
 * nothing carried over from earlier E-steps (their scheduling costs and store
 * sizes); the next hmc_em_iteration(1, ..., *old_ll = -DBL_MAX) starts a fresh
 * chain.  Results equal a fresh context's.  After a rewind, hmc_get_patterns
 * spells whole allele strings only if no table was mined since the save (the
 * candidate tree that spells them is not kept); otherwise the last allele. */
int hmc_model_save(hmc_ctx *ctx);
int hmc_em_rewind(hmc_ctx *ctx);
/* HaploComp (HaploComp.cpp:29-155) of the input panel, phase as given,
 * against the accepted resolutions: switch error, incorrect-haplotype and
 * incorrect-genotype percentages over all ranks' individuals.  Replaces the
 * HaploComp compare(&genos, &resolutions) of HaploModel.cpp:134. */
int hmc_haplocomp(hmc_ctx *ctx, double *switch_error, double *ihp, double *igp);
/* Accepted resolutions of the last hmc_run ([n][2][L] symbols). */
int hmc_get_best_resolutions(hmc_ctx *ctx, int32_t *out);
/* HaploFile::writeGenoData (HaploFile.cpp:120-153) of the accepted
 * resolutions (single-rank contexts): the loaded file's positions ("P" line)
 * and ids ('#' prepended only to an id starting with a digit), or the
 * defaults k*1000 and 1..N for a panel loaded from memory. */
int hmc_write_phase(hmc_ctx *ctx, const char *path);
/* HaploFile::getHaploFile(format, file names) + readGenoData / writeGenoData
 * (HaploFile.cpp:13-52, 54-153, 205-640).  format / file names:
 *   "PHASE", "HPM", "HPM2"  one file;
 *   "BENCH2"                genotype file, position file;
 *   "BENCH3"                genotype file, position file, children file — the
 *                           children are appended as ordinary unphased
 *                           genotypes, unphased_num = the parents, and HaploComp
 *                           covers the parents only (HaploFile.cpp:446-484,
 *                           HaploComp.cpp:40).
 * hmc_parse_files needs no context or device: it returns the panel (alleles
 * [N][2][L] symbols, -1 missing; types [L+1] 'S'/'M'; unphased_num); pass NULL
 * buffers first to learn N and L.  hmc_load_files = parse + hmc_load_genotypes
 * (keeps ids, marker names, positions for the writers).  hmc_write_files
 * writes the accepted resolutions in that format (BENCH2/3: genotype file +
 * position file). */
int hmc_parse_files(const char *format, const char *const *paths, int n_paths, int *N, int *L, int32_t *alleles,
                    char *types, int *unphased_num);
int hmc_load_files(hmc_ctx *ctx, const char *format, const char *const *paths, int n_paths);
int hmc_write_files(hmc_ctx *ctx, const char *format, const char *const *paths, int n_paths);
/* GenoData::unphased_num (GenoData.h:37) of the loaded panel. */
int hmc_unphased_num(const hmc_ctx *ctx, int *unphased_num);
/* One- and two-file shorthands of the three calls above (path2 may be NULL). */
int hmc_parse_file(const char *format, const char *path, const char *path2, int *N, int *L, int32_t *alleles,
                   char *types);
int hmc_load_file(hmc_ctx *ctx, const char *format, const char *path, const char *path2);
int hmc_write_file(hmc_ctx *ctx, const char *format, const char *path, const char *path2);
/* HaploFile::writePattern (HaploFile.cpp:155-171; HMC.cpp:229-232, the
 * --output-patterns ".patterns" file) of the current pattern table: header
 * "Frequency\tLength\t<marker names>", one line per pattern in id order with
 * frequency / N, length and the long-format alleles (-1 outside the pattern).
 * The reference divides by genotype_num() of a GenoData that no longer exists
 * when it writes, so the N used here is the panel's: unpinned. */
int hmc_write_patterns(hmc_ctx *ctx, const char *path);

/* ---- tuning -------------------------------------------------------------- */
/* frontier_cap: initial states per locus and individual (doubles on
 * overflow, at most 2 097 151); trace_bytes: trace-store budget (0 =
 * automatic); waves: resident E-step waves (0 = automatic). */
int hmc_set_tuning(hmc_ctx *ctx, int frontier_cap, uint64_t trace_bytes, int waves);
/* E-step launch shape: wavefronts cooperating on one individual (1..4,
 * default 2) and individuals sharing one CU's LDS (default 8); 0 keeps the
 * current value.  A shape set here applies to every kernel; (0, 0) returns the
 * split E-step's value pass to its automatic shape: 1 wave x 20 individuals per
 * CU for groups of at least 32 individuals per CU, 2 x 8 from 8 per CU, else
 * 3 x 8; a value-pass shape given by one number only takes the other from the
 * same rule.  Results do not depend on the shape. */
int hmc_set_estep_shape(hmc_ctx *ctx, int waves_per_individual, int individuals_per_cu);
/* Launch shapes of the split E-step's two passes, 0 = automatic for each:
 * structure pass waves per individual (1, 4, 8 or 16; automatic: 4 on a model
 * with more patterns than the panel has individual-loci, the genotype-mined
 * M0, 16 when such a group has at most one individual per CU)
 * and individuals per CU (automatic: 1 at 16 waves, 2 at 4; else 12 above 8 per CU in
 * the group, 8 above 4, else 4), value pass waves per individual (1..4) and
 * individuals per CU (rule of hmc_set_estep_shape; groups averaging more than
 * 1 500 record words per locus take 8 x 2, or 16 / c waves x c per CU when
 * they have c < 4 individuals per CU).  Value-pass waves per individual 1..16.
 * Results do not depend on them. */
int hmc_set_pass_shapes(hmc_ctx *ctx, int structure_waves, int structure_ipc, int value_waves, int value_ipc);
/* Budgets of the split E-step's two stores in bytes, 0 = automatic: the
 * k-best trace store (min(42 % of free HBM, 120 GiB)) and the structure-record
 * store (min(28 %, 80 GiB); 0 with a trace budget given = the same number).
 * Individuals pass in groups whose records and traces fit them. */
int hmc_set_store_budgets(hmc_ctx *ctx, uint64_t trace_bytes, uint64_t record_bytes);
/* E-step implementation: 0 (default) = two passes, a structure pass that
 * replays extendAll/addHaploPair (HaploBuilder.cpp:226-261) on pattern ids
 * and a value pass with the k-best lists; individuals whose forward
 * likelihood underflows are re-run through a structure pass that applies
 * extend()'s forward test (HaploBuilder.cpp:237); 1 = the fused single-pass
 * kernel (sample_size <= 32).  Both produce identical results. */
int hmc_set_estep_mode(hmc_ctx *ctx, int mode);
/* Split E-step of the last hmc_resolve_all: device ms of the structure pass,
 * the value pass and the underflow re-runs, and the number of individuals
 * re-run. */
int hmc_last_estep_split(const hmc_ctx *ctx, double *structure_ms, double *values_ms, double *fallback_ms,
                         int *n_fallback);
/* Launches of the last hmc_resolve_all: structure passes and value passes
 * (individuals pass in groups when their records / traces exceed the stores). */
int hmc_last_estep_passes(const hmc_ctx *ctx, int *structure_passes, int *value_passes);
/* Value pass of the split E-step.  Mode 0: k-best lists are kept by
 * likelihood value only; an individual for which that could change a result
 * (a non-zero likelihood tied across some list's S-cut — the set
 * std::nth_element keeps then depends on the list order, HaploPair.cpp:85-88 —
 * or final candidates with equal or zero priors, HaploBuilder.cpp:101-105) is
 * re-run with the libstdc++ permutations.  Mode 1: every individual with the
 * libstdc++ permutations.  Mode 2 (default): automatic — mode 0 on panels with
 * more than two alleles per locus once the model is smaller than the panel,
 * mode 1 otherwise and for the rest of the context once a mode-0 E-step
 * re-ran more than 35 % of its individuals.  Results are identical in every
 * mode; mode 0 pays off only where few individuals have such ties (at
 * BASELINE config 3 about half of them have final candidates with equal
 * priors, and mode 1 is faster; at config 5's later E-steps a quarter). */
int hmc_set_value_mode(hmc_ctx *ctx, int mode);
/* Phase-B layout of the value pass (results identical): the overflowing adds'
 * selections with two links per lane (S lanes and 64 / S lists per
 * wavefront, sample_size <= 16) instead of one (2S lanes, 64 / 2S lists).
 * Mode 0: never; 1: groups of heavy individuals (the first E-step on a
 * genotype-mined model: many chains of adds per locus); 2 (default): every
 * group. */
int hmc_set_value_layout(hmc_ctx *ctx, int mode);
/* Schedule of the value pass (results identical): 1 = locus by locus (every
 * state's constructor and appends, a block barrier, the chains of adds, a
 * barrier); 2 = dataflow (one wavefront builds the lists in locus order as
 * soon as a state's predecessors are final, the others run the chains of
 * adds of any open locus; `ring` = frontiers kept, 3 or 4, 0 = 3); 0
 * (default) = automatic.  The same HaploPair::add sequence per state
 * (HaploPair.cpp:35-89) either way. */
int hmc_set_value_pass(hmc_ctx *ctx, int mode, int ring);
/* Structure pass of the split E-step (results identical): 1 = per chunk of
 * contributions a ranking hand-off (lane masks, four block barriers per
 * chunk); 2 = three block scans per locus (creation order from each key's
 * first contribution, add order from each state's member segment); 0 =
 * automatic. */
int hmc_set_structure_pass(hmc_ctx *ctx, int version);
/* Dataflow value pass: wavefronts per individual that build the lists which
 * need no selection (the "A" waves, each a fixed share of every locus's
 * states), 1..8 and fewer than the waves per individual; 0 = by the launch
 * shape.  Results are identical. */
int hmc_set_dataflow_waves(hmc_ctx *ctx, int a_waves);
/* Structure pass over the pattern table in end-locus order (1, default) or
 * in the table's id order (0): the successor lookups of one locus fall in one
 * block of the table instead of lines spread over all of it.  Results are
 * identical. */
int hmc_set_end_order(hmc_ctx *ctx, int on);
/* Exact M-step trie walk (HaploBuilder.cpp:334-449 estimateFrequency): 0 or
 * 1 = the depth-first walk, one (individual, start locus) item per wavefront
 * (default); 4 = four items per wavefront (16 lanes each) and 2 = the
 * breadth-first walk, one trie node per lane (both measured slower: the
 * variants library only, HMC_EUNSUPPORTED in the product).  The frequency
 * sums are fixed-point integer adds, identical for any order. */
int hmc_set_exact_walk(hmc_ctx *ctx, int items_per_wave);
/* 1 when the last value-pass launch ran the dataflow schedule. */
int hmc_last_value_pass(const hmc_ctx *ctx, int *dataflow);
/* Windowed E-step (SURVEY §7 hard part 4): the loci in windows, each
 * window's last frontier saved as the next one's checkpoint; records are kept
 * for one window and full traces for two, the older one collected into
 * survivor nodes (the entries the traceback can still reach).  Results are
 * identical to the classic passes.  mode 0 (default): automatic — when the
 * first loci of a sample show that the classic passes could hold fewer than
 * two individuals per CU in a group (cfg 4's per-rank E1) or would need three
 * or more groups (cfg 3's E1); 1 never; 2 always (tests).  window_loci: loci
 * per window (0: from the store budgets).
 * Replaces no reference interface (HaploBuilder::resolve keeps every locus's
 * pairs alive, HaploBuilder.cpp:35-126). */
int hmc_set_estep_windows(hmc_ctx *ctx, int mode, int window_loci);
/* The last E-step's windows (0 = classic passes), loci per window, groups of
 * individuals, and device ms of the trace collections (part of the value
 * passes' time). */
int hmc_last_estep_windows(const hmc_ctx *ctx, int *windows, int *window_loci, int *groups, double *recompute_ms);
/* Restarts of the last E-step (a frontier or contribution capacity grown, or
 * a window's traces past the store: windows 0.6x as long, or for a fixed
 * window length smaller groups) and the window scale now in force (1.0 until
 * a trace-store overflow; reset by a panel load or hmc_set_shard). */
int hmc_last_estep_restarts(const hmc_ctx *ctx, int *restarts, double *window_scale);
/* Host wall time (ms) of the last hmc_em_iteration's phases, in this order:
 * [0] the E-step call, [1] its store (re)allocations and releases, [2] the
 * end-order table build, [3] the sample gather after the passes, [4] accepting
 * the resolutions, [5] HaploComp, [6] the M-step call, [7] the E-step's setup
 * before the passes (buffers, budgets, cost order).  [1]-[3] and [7] are parts
 * of [0].  Writes min(n, 8) values and returns 8.  Replaces no reference
 * interface (measurement of the per-rank host gap). */
int hmc_last_host_phases(const hmc_ctx *ctx, double *ms, int n);
/* Individuals the last E-step re-ran with the libstdc++ permutations (mode 0)
 * and the device time of those re-runs (ms, part of values_ms). */
int hmc_last_estep_order(const hmc_ctx *ctx, int *n_rerun, double *rerun_ms);
/* Device time (ms, HIP events on the context stream) of the last E-step
 * forward kernel, traceback and whole M-step. */
int hmc_last_timings(const hmc_ctx *ctx, double *estep_forward_ms, double *estep_traceback_ms, double *mstep_ms);

/* ---- CPU-side test hooks (no GPU needed) --------------------------------- */
/* The libstdc++-exact selection used by the E-step kernel (select.hpp), run on
 * host arrays: nth_element(v, v+nth, v+n, greater) and sort(v, v+n, greater)
 * of (lik, tag) records ordered by lik. */
void hmc_test_nth_element(double *lik, uint32_t *tag, int n, int nth);
void hmc_test_sort_small(double *lik, uint32_t *tag, int n);
/* std::sort(v, v+n, greater) for any n (introsort, heap sort at depth 0,
 * final insertion sort): the final candidate order for sample_size > 16. */
void hmc_test_sort(double *lik, uint32_t *tag, int n);
/* The E-step's mask-partition formulation of the same nth_element (n <= 32). */
void hmc_test_nth_element_masks(double *lik, uint32_t *tag, int n, int nth);
/* GPU check of the segmented wave selection the E-step kernel uses
 * (coop_select.hpp), 64/seg_width lists per wavefront: list b =
 * lik/tag[off[b] .. off[b]+n[b]) (n[b] <= seg_width <= 32) gets
 * nth_element(.., nth[b], greater) in place on `device`. */
int hmc_test_coop_nth_element(int device, double *lik, uint32_t *tag, const int32_t *off, const int32_t *n,
                              const int32_t *nth, int count, int total, int seg_width);
/* Library version string. */
const char *hmc_version(void);
/* Version, target, flags and build time of this libhmc_amd.so (bench.py
 * prints it with the path of the library it loaded). */
const char *hmc_build_info(void);
/* Environment read by the library (diagnostics only; none changes a result
 * or what runs): HMC_DEBUG_MEM, HMC_DIAG_MINE print E-step group / mining
 * statistics to stderr; HMC_FORCE_COLLECTIVES makes a one-rank context run
 * its RCCL collectives anyway (test hook). */

#ifdef __cplusplus
}
#endif
#endif /* HMC_AMD_H */
