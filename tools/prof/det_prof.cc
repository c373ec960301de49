// Host result-chain profiling (development; not part of the library): the
// lattices of tools/prof/det_dump.py through prune, pruned phone + word
// determinization, graph scale, word alignment and MBR, repeated; built by
// tools/prof/Makefile with -pg for gprof.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "../../vosk-api_amd/csrc/lattice.h"
#include "../../vosk-api_amd/csrc/model_io.h"

using namespace vamd;

template <class T>
static std::vector<T> rd(std::ifstream& f) {
  long long n = 0;
  f.read((char*)&n, 8);
  std::vector<T> v(n);
  f.read((char*)v.data(), sizeof(T) * n);
  return v;
}

int main(int argc, char** argv) {
  std::ifstream f(argv[1], std::ios::binary);
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  Graph g;
  g.ilabel = rd<int>(f);
  g.olabel = rd<int>(f);
  std::vector<int> tid2phone = rd<int>(f);
  std::vector<char> tid_first = rd<char>(f), ty = rd<char>(f), fi = rd<char>(f), lo = rd<char>(f);
  long long n = 0;
  f.read((char*)&n, 8);
  std::vector<RawLattice> lats(n);
  for (auto& L : lats) {
    long long nf = 0;
    f.read((char*)&nf, 8);
    L.num_frames = (int)nf;
    std::vector<int> fb = rd<int>(f), ts = rd<int>(f);
    std::vector<float> tc = rd<float>(f);
    std::vector<int> ls = rd<int>(f), ld = rd<int>(f), la = rd<int>(f);
    std::vector<float> lg = rd<float>(f), lx = rd<float>(f), fc = rd<float>(f);
    L.frame_begin = fb;
    L.tok_state = ts;
    L.tok_cost = tc;
    for (size_t i = 0; i < ls.size(); i++) L.links.push_back(RawLattice::Link{ls[i], ld[i], la[i], lg[i], lx[i]});
    L.final_cost = fc;
  }
  double t[4] = {0, 0, 0, 0};
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  for (int r = 0; r < reps; r++)
    for (const RawLattice& L0 : lats) {
      RawLattice L = L0;
      LatticeOptions opt;
      opt.lattice_beam = 6.0f;
      const auto t0 = clk::now();
      PruneRawLattice(&L, 6.0f);
      WordLattice wl;
      DeterminizePhonePruned(L, g, tid2phone, tid_first, opt, &wl);
      const auto t1 = clk::now();
      ScaleGraph(&wl, 0.9f);
      WordLattice al;
      WordAlignLattice(wl, ty, fi, lo, 1000000, &al);
      const auto t2 = clk::now();
      MbrResult m;
      MinimumBayesRisk(al, &m);
      const auto t3 = clk::now();
      t[0] += ms(t0, t1);
      t[1] += ms(t1, t2);
      t[2] += ms(t2, t3);
    }
  const double k = 1.0 / (reps * (double)n);
  printf("per segment: determinize %.3f ms, align %.3f ms, mbr %.3f ms\n", t[0] * k, t[1] * k, t[2] * k);
  return 0;
}
