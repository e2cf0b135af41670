"""Chain statistics of the E-step on the CPU restatement (diagnostic, never the
product): the oracle (oracle/hmc_oracle.cpp) is copied to a temporary
directory, instrumented around HaploPair::add (its nth_element calls) and
built there; the repository's oracle is not touched.

Per individual-locus: states, chains (states whose adds overflow S), adds, the
longest chain, steps with 3 / 24 segments; histograms of chain lengths; and
per individual the dataflow critical path (a state's add waits only for its
own predecessor's list) against the per-locus sum of longest chains.

    python tools/diag/chain_stats.py CFG [N_SAMPLE]   (N_SAMPLE > 0: E1 only, on a
                                                      sample spread over the panel)
"""
import ctypes as C
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

PATCHES = [
    ("struct Model {", """uint64_t g_st[8]; uint64_t g_hist_len[64]; uint64_t g_hist_max[64]; uint64_t g_df[4];
static thread_local std::vector<int> st_calls;
static thread_local std::vector<double> fin_cur, fin_nxt;  // dataflow finish time per state
static thread_local double barrier_time;
struct Model {"""),
    ("""      nxt.push_back(std::move(x));
      best[key] = (int)nxt.size();""", """      nxt.push_back(std::move(x));
      best[key] = (int)nxt.size();
      if ((int)fin_nxt.size() < (int)nxt.size()) fin_nxt.resize(nxt.size(), 0.0);
      fin_nxt[nxt.size() - 1] = predIdx < (int)fin_cur.size() ? fin_cur[predIdx] : 0.0;"""),
    ("""      if ((int)x.links.size() > S) {
        std::nth_element(x.links.begin(), x.links.begin() + S - 1, x.links.end(), GreaterLik());""",
     """      { double pf = predIdx < (int)fin_cur.size() ? fin_cur[predIdx] : 0.0; double &f = fin_nxt[it->second - 1];
        f = f > pf ? f : pf; if ((int)x.links.size() > S) f += 1.0; }
      if ((int)x.links.size() > S) {
        if ((int)st_calls.size() <= it->second) st_calls.resize(it->second + 1, 0);
        st_calls[it->second - 1]++;
        std::nth_element(x.links.begin(), x.links.begin() + S - 1, x.links.end(), GreaterLik());"""),
    ("""      uni_check((int)hp[i + 1].size());""", """      uni_check((int)hp[i + 1].size());
      { int nch = 0, tot = 0, mx = 0; int ns = (int)hp[i + 1].size();
        for (int q = 0; q < ns && q < (int)st_calls.size(); ++q) { int c = st_calls[q];
          if (c) { nch++; tot += c; if (c > mx) mx = c; __atomic_fetch_add(&g_hist_len[c < 63 ? c : 63], 1, __ATOMIC_RELAXED); }
          st_calls[q] = 0; }
        __atomic_fetch_add(&g_st[0], (uint64_t)nch, __ATOMIC_RELAXED); __atomic_fetch_add(&g_st[1], (uint64_t)tot, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_st[2], (uint64_t)mx, __ATOMIC_RELAXED); __atomic_fetch_add(&g_st[3], (uint64_t)1, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_st[4], (uint64_t)ns, __ATOMIC_RELAXED);
        int t3 = (tot + 2) / 3; __atomic_fetch_add(&g_st[5], (uint64_t)(t3 > mx ? t3 : mx), __ATOMIC_RELAXED);
        int t24 = (tot + 23) / 24; __atomic_fetch_add(&g_st[6], (uint64_t)(t24 > mx ? t24 : mx), __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_hist_max[mx < 63 ? mx : 63], 1, __ATOMIC_RELAXED);
        barrier_time += mx; fin_cur.assign(fin_nxt.begin(), fin_nxt.begin() + ns); fin_nxt.clear(); }"""),
    ("""    hp.assign(L + 1, {});
    tie_cur = 0;""", """    hp.assign(L + 1, {});
    tie_cur = 0;
    fin_cur.assign(4096, 0.0); fin_nxt.clear(); barrier_time = 0;"""),
    ("""    uint64_t re = 0;
    for (int i = hl; i <= L; ++i)""", """    { double cp = 0; for (double f : fin_cur) cp = f > cp ? f : cp;
      __atomic_fetch_add(&g_df[0], (uint64_t)(cp * 1000), __ATOMIC_RELAXED);
      __atomic_fetch_add(&g_df[1], (uint64_t)(barrier_time * 1000), __ATOMIC_RELAXED);
      __atomic_fetch_add(&g_df[2], (uint64_t)1, __ATOMIC_RELAXED); }
    uint64_t re = 0;
    for (int i = hl; i <= L; ++i)"""),
    ('extern "C" {', '''extern "C" {
void ora_chain_stats(uint64_t *o) {
  for (int i = 0; i < 8; i++) { o[i] = ora::g_st[i]; ora::g_st[i] = 0; }
  for (int i = 0; i < 64; i++) { o[8 + i] = ora::g_hist_len[i]; o[72 + i] = ora::g_hist_max[i]; ora::g_hist_len[i] = ora::g_hist_max[i] = 0; }
  for (int i = 0; i < 4; i++) { o[136 + i] = ora::g_df[i]; ora::g_df[i] = 0; }
}
'''),
]


def build(tmp):
    src = open(os.path.join(ROOT, "oracle", "hmc_oracle.cpp")).read()
    for old, new in PATCHES:
        assert old in src, old[:60]
        src = src.replace(old, new, 1)
    open(os.path.join(tmp, "hmc_oracle.cpp"), "w").write(src)
    shutil.copy(os.path.join(ROOT, "oracle", "oracle.py"), tmp)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-fPIC", "-pthread", "-ffp-contract=off", "-shared", "-o",
                           os.path.join(tmp, "liboracle.so"), os.path.join(tmp, "hmc_oracle.cpp")])


def report(L, tag):
    s = (C.c_uint64 * 140)()
    L.ora_chain_stats(s)
    s = list(s)
    nl, n = max(s[3], 1), max(s[138], 1)
    print(f"{tag}: individual-loci {s[3]} states/locus {s[4] / nl:.1f} chains/locus {s[0] / nl:.2f} "
          f"adds/locus {s[1] / nl:.2f} longest chain/locus {s[2] / nl:.2f} steps(3 segments) {s[5] / nl:.2f} "
          f"steps(24 segments) {s[6] / nl:.2f}")
    print(f"   per individual: dataflow critical path {s[136] / 1000 / n:.1f} adds, per-locus longest chains "
          f"{s[137] / 1000 / n:.1f} adds, ratio {s[137] / max(s[136], 1):.2f}")
    print("   chain lengths", {i: s[8 + i] for i in range(64) if s[8 + i]})
    print("   longest chain per locus", {i: s[72 + i] for i in range(64) if s[72 + i]}, flush=True)


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sample = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    tmp = tempfile.mkdtemp(prefix="chain_stats_")
    build(tmp)
    sys.path.insert(0, tmp)
    import oracle
    from hmc_amd import synth

    oracle.set_threads(os.cpu_count() or 1)
    L = oracle.lib()
    L.ora_chain_stats.argtypes = [C.POINTER(C.c_uint64)]
    p = synth.config_panel(cfg)
    o = oracle.Oracle(p.alleles, p.types, sample_size=10, max_iter=1)
    o.find_patterns()
    report(L, "M0 (discard)")
    if sample:
        o.time_resolve_list(np.linspace(0, p.N - 1, sample).astype(int).tolist())
        report(L, f"cfg {cfg} E1 ({sample} individuals)")
        return
    for it in range(3):
        o.resolve_all()
        report(L, f"cfg {cfg} E{it + 1}")
        o.find_patterns()


if __name__ == "__main__":
    main()
