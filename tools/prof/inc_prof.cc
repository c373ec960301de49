// Host profiling of the KaldiRecognizer's incremental lattice (development;
// not part of the library): the records of tools/prof/inc_dump.py replayed
// through IncrementalLattice (AdvanceDecoding ends, FinalizeDecoding, the
// final GetLattice) three times, with the phase timers of incremental.cc.
// Built by tools/prof/Makefile (inc_prof).
#include <cstdio>
#include <vector>
#include <chrono>
#include <string>
#include "incremental.h"
#include "model_io.h"
using namespace vamd;

static FILE* F;
template <class T> std::vector<T> rd() {
  long long n = 0;
  if (fread(&n, 8, 1, F) != 1) return {};
  std::vector<T> v(n);
  if (n && fread(v.data(), sizeof(T), n, F) != (size_t)n) v.clear();
  return v;
}
int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: inc_prof records.bin\n"); return 1; }
  F = fopen(argv[1], "rb");
  if (!F) return 1;
  Graph g; g.ilabel = rd<int>(); g.olabel = rd<int>(); g.weight = rd<float>(); g.final_cost = rd<float>(); g.start = rd<int>()[0];
  auto t2p = rd<int>(); auto tf8 = rd<signed char>(); std::vector<char> tf(tf8.begin(), tf8.end());
  int nf = rd<int>()[0];
  struct Fr { std::vector<int> st; std::vector<float> co; float off; std::vector<IncFrameIn::Link> ln; };
  std::vector<Fr> fr(nf);
  for (int k = 0; k < nf; k++) {
    fr[k].st = rd<int>(); fr[k].co = rd<float>(); fr[k].off = rd<float>()[0];
    auto L = rd<int>(); auto A = rd<float>();
    for (size_t i = 0; i < A.size(); i++) fr[k].ln.push_back(IncFrameIn::Link{L[3*i], L[3*i+1], L[3*i+2], A[i], false});
    for (auto& l : fr[k].ln) l.emit = g.ilabel[l.arc] != 0;
  }
  auto et = rd<int>(), ea = rd<int>();
  IncrementalOptions o;
  for (int rep = 0; rep < 3; rep++) {
    for (double& x : vamd_inc_prof) x = 0;
    IncrementalLattice inc; inc.Init(&g, &t2p, &tf, o);
    auto t0 = std::chrono::steady_clock::now();
    for (size_t e = 0; e < et.size(); e++) {
      if (et[e] == 0) {
        while (inc.NumFramesDecoded() < ea[e]) { int k = inc.NumFramesDecoded() + 1; IncFrameIn f; f.state = fr[k].st.data(); f.cost = fr[k].co.data(); f.ntok = fr[k].st.size(); f.cost_offset = fr[k].off; f.links = fr[k].ln.data(); f.nlinks = fr[k].ln.size(); inc.AddFrame(f); }
        inc.AdvanceEnd();
      } else { inc.FinalizeDecoding(); WordLattice wl; inc.GetLattice(inc.NumFramesDecoded(), true, &wl); printf("states %d\n", wl.NumStates()); }
    }
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("total %.1f ms: add %.1f prune %.1f build %.1f det %.1f accept %.1f\n", ms, vamd_inc_prof[0], vamd_inc_prof[1], vamd_inc_prof[2], vamd_inc_prof[3], vamd_inc_prof[4]);
  }
}

namespace vamd {
void LogMessage(const char*, const std::string&) {}
}
