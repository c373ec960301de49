// Lattices of the decoder's segment (host side).
//
// The decode kernel keeps Kaldi's forward links (LatticeFasterDecoder /
// LatticeIncrementalDecoder [K]; the reference builds its results from the
// decoder's lattice, src/recognizer.cc:669-729 GetResult -> MbrResult /
// NbestResult / NlsmlResult, and src/batch_recognizer.cc:43-107) in HBM per
// stream: raw relaxations, LatFrame records and the token arena
// (engine_dev.h).  RawLattice is the canonical state-level lattice built from
// them (GetRawLattice): tokens per frame, deduplicated links below each
// frame's cutoff, graph / acoustic costs, final costs.  The word-level steps
// (lattice-beam pruning, determinization, MBR) live in lattice.cc.
#pragma once
#include <algorithm>
#include <cstdint>
#include <limits>
#include <string>
#include <utility>
#include <vector>

#include <hip/hip_runtime.h>

#include "engine_dev.h"

namespace vamd {

struct Graph;
struct TransitionTables;

struct RawLattice {
  int num_frames = 0;                // decoded frames; token frames are 0..num_frames
  std::vector<int> frame_begin;      // [num_frames + 2] tokens of frame k: [frame_begin[k], frame_begin[k+1])
  std::vector<int> tok_state;
  std::vector<float> tok_cost;       // decoder tot_cost (with the frames' cost offsets)
  struct Link {
    int src, dst;                    // token ids
    int arc;                         // graph arc (ilabel = transition-id or 0, olabel = word or 0)
    float graph_cost;                // arc weight
    float acoustic_cost;             // decoder's ac cost minus the frame's cost offset (0 for epsilon)
  };
  std::vector<Link> links;           // sorted by (destination frame, src, arc)
  std::vector<float> final_cost;     // per token of the last frame (+inf: not final); empty = all final with 0
  bool overflow = false;             // link arena / frame table overflowed: incomplete
  int FrameOf(int tok) const {
    return (int)(std::upper_bound(frame_begin.begin(), frame_begin.end(), tok) - frame_begin.begin()) - 1;
  }
};

// Canonical lattice from the device records of one stream: frames [0, F]
// (LatFrame), the token arena {prev, arc, cost, state} and the frames'
// links {src, dst arena index, arc, acoustic cost} (engine_dev.h; the
// decoder already keeps exactly Kaldi's links).  Dead arena entries
// (prev == -2) are skipped; links are sorted by (source, arc) per frame.
// use_final: final costs of the last frame's tokens if any token is final
// (Kaldi GetRawLattice with use_final_probs).
void BuildRawLattice(const Graph& g, int start_state, const std::vector<LatFrame>& frames,
                     const std::vector<int4>& arena, const std::vector<int4>& links,
                     bool use_final, RawLattice* out);

// ---- word level (lattice.cc)

// A word lattice after determinization: states topologically sorted (0 =
// start), every arc one word (0 = epsilon word), weight = (graph, acoustic)
// pair, and the transition-ids of the frames the arc spans.
struct WordLattice {
  struct Arc {
    int word, next;
    float graph, acoustic;
    std::vector<int> tids;
  };
  std::vector<std::vector<Arc>> arcs;
  std::vector<float> final_graph, final_acoustic;  // +inf graph: not final
  std::vector<std::vector<int>> final_tids;
  int NumStates() const { return (int)arcs.size(); }
};

struct LatticeOptions {
  float lattice_beam = 6.0f;  // also the pruned determinization's beam (GetLattice)
  int max_states = 100000;  // determinization guard (falls back to the best path)
  long long det_max_mem = 50000000;  // DeterminizeLatticePhonePrunedOptions::max_mem [K]
};

// Lattice-beam pruning of the raw lattice (PruneForwardLinks /
// PruneForwardLinksFinal semantics: keep links and tokens whose best path
// through them is within lattice_beam of the best complete path).
void PruneRawLattice(RawLattice* lat, float lattice_beam);

// Word-level determinization (DeterminizeLatticePruned [K]): one path per
// word sequence, the best alignment, strings output as their common prefix.
// Returns false if the guard tripped.
bool DeterminizeToWords(const RawLattice& lat, const Graph& g, const LatticeOptions& opt,
                        WordLattice* out);

// Kaldi's DeterminizeLatticePhonePrunedWrapper, the determinization of the
// reference's GetLattice (src/recognizer.cc:678; batch lattices through the
// CUDA pipeline's determinize step): a phone label inserted at the first
// transition-id of every phone (tid_first: HMM state 0, not a self-loop),
// determinization on phones + words, the result expanded back to a
// one-transition-id-per-link lattice with the phone labels deleted, then
// word-level determinization of that.  Both passes are Kaldi's pruned
// determinization (LatticeDeterminizerPruned at beam lattice_beam: best-first
// transitions within the beam, max_mem with the narrower-beam retry; see
// lattice.cc).  False if a guard tripped.
bool DeterminizePhonePruned(const RawLattice& lat, const Graph& g, const std::vector<int>& tid2phone,
                            const std::vector<char>& tid_first, const LatticeOptions& opt, WordLattice* out);

// The determinizer's input: an acceptor on `lout` (words, or phones in the
// first pass; any label above the words -- the incremental determinizer's
// state and token labels -- is a word to it) whose links carry one
// transition-id (`lin`, 0 = none) as the string side: Kaldi's Lattice after
// Invert (DeterminizeLatticePhonePrunedWrapper).  frame: per state, a bucket
// such that every link goes to the same or a later bucket (the closure's work
// order).  LW: a LatticeWeight (graph, acoustic).
struct LW {
  float g = 0.0f, a = 0.0f;
};
struct DetGraph {
  int n = 0, start = -1;
  std::vector<int> frame;
  struct Link {
    int src, dst, lin, lout;
    float g, a;
  };
  std::vector<Link> links;
  std::vector<LW> fin;  // +inf graph: not final
  int AddState(int f) {
    frame.push_back(f);
    fin.push_back(LW{std::numeric_limits<float>::infinity(), 0.0f});
    return n++;
  }
};
// DeterminizePhonePruned on a determinizer input built by the caller (the
// start state's links get no phone label, as DeterminizeLatticeInsertPhones).
bool DeterminizePhonePrunedGraph(DetGraph D, const std::vector<int>& tid2phone, const std::vector<char>& tid_first,
                                 const LatticeOptions& opt, WordLattice* out);

// Word alignment (Kaldi lat/word-align-lattice.cc WordAlignLattice [K], with
// WordBoundaryInfo from word_boundary.int and reorder = true; the reference
// aligns before MBR and n-best, src/recognizer.cc:433-434,555-558,
// src/batch_recognizer.cc:48): every output arc spans exactly one word (begin
// .. end phone, or a singleton phone) or one non-word phone (word 0), the
// word label moved onto its phones.  Per-state pending transition-ids and
// word labels (the aligner's computation state), advance weights on epsilon
// transitions removed at the end (RmEpsilon).  phone_type per phone: 1
// nonword, 2 begin, 3 end, 4 internal, 5 singleton.  False if the guard trips.
bool WordAlignLattice(const WordLattice& in, const std::vector<char>& tid2phone_type,
                      const std::vector<char>& tid2final, const std::vector<char>& tid2selfloop,
                      int max_states, WordLattice* out);

// Scale the graph part of every weight (fst::GraphLatticeScale, src/recognizer.cc:718)
void ScaleGraph(WordLattice* lat, float scale);

// Minimum Bayes risk decoding (Kaldi lat/sausages.cc MinimumBayesRisk [K]):
// one-best words, their confidences (posteriors in the aligned bins) and
// times (frames, from the bin averages).
struct MbrResult {
  std::vector<int> words;
  std::vector<float> conf;
  std::vector<std::pair<float, float>> times;
};
void MinimumBayesRisk(const WordLattice& lat, MbrResult* out);

// n-best distinct word sequences (fst::ShortestPath on the determinized
// lattice, src/recognizer.cc:484-607): words, per-word frame spans, total
// cost split into (graph, acoustic).
struct NbestPath {
  std::vector<int> words;
  std::vector<std::pair<int, int>> spans;  // [begin, end) frames of each word
  float graph = 0, acoustic = 0;
};
void NbestPaths(const WordLattice& lat, int n, std::vector<NbestPath>* out);

}  // namespace vamd
