// LM rescoring of a segment's word lattice.
//
// Reference: src/model.cc:308-314 loads rescore/G.fst (ReadAndPrepareLmFst:
// projected on its output labels when it is not an acceptor, ilabel-sorted)
// and rescore/G.carpa (Kaldi ConstArpaLm); src/recognizer.cc:675-711 takes the
// decoder's determinized lattice, subtracts the old LM (graph costs negated,
// composed with G, determinized on words, negated back) and adds the ConstArpa
// LM by deterministic composition, before the graph scale and the MBR /
// n-best result.  RNNLM rescoring (rescore/../rnnlm) is not implemented.
//
// Host-side lattice work on the segment's (small) word lattice: the GPU keeps
// the state-level lattice; rescoring runs once per final result.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "lattice.h"
#include "model_io.h"

namespace vamd {

// Kaldi lm/const-arpa-lm.{h,cc} [K] binary object: "<ConstArpaLm>" with
// <LmInfo> (bos, eos, unk, order), <LmStates> (int32 array: per history
// [logprob][backoff logprob][num children][(word, child info) x n], children
// sorted by word; child info even = the leaf n-gram's logprob bits, odd =
// 2 * relative offset + 1 of the child's history state, negative offsets
// index the overflow table), <LmUnigram> (int64 offset of each word's
// unigram state, 0 = none) and <LmOverflow>.  Natural-log probabilities.
class ConstArpaLm {
 public:
  void Read(const std::string& path);
  // GetNgramLogprob: backoff over the history (oldest word first), unknown
  // words mapped to <unk> when the LM has one; -inf when unknown
  float NgramLogprob(int word, std::vector<int> hist) const;
  bool HistoryStateExists(const std::vector<int>& hist) const;
  int bos = -1, eos = -1, unk = -1, order = 0;

 private:
  const int32_t* UnigramState(int w) const;
  const int32_t* State(const std::vector<int>& seq) const;
  bool ChildInfo(int word, const int32_t* parent, int32_t* info) const;
  void Decode(int32_t info, const int32_t* parent, const int32_t** child, float* logprob) const;
  float Recurse(int word, const std::vector<int>& hist) const;
  std::vector<int32_t> states_;
  std::vector<int64_t> unigram_, overflow_;
};

struct RescoreLm {
  HostFst g;          // the LM to subtract (acceptor, ilabel-sorted)
  ConstArpaLm carpa;  // the LM to add
  void Load(const std::string& g_fst, const std::string& g_carpa);
};

// The rescored lattice of a determinized word lattice (graph costs
// unscaled); false (and a warning) if it comes out empty or the guard trips.
bool RescoreLattice(const WordLattice& in, const RescoreLm& lm, const LatticeOptions& opt,
                    WordLattice* out);

}  // namespace vamd
