// The KaldiRecognizer's lattice: Kaldi's LatticeIncrementalDecoder token
// bookkeeping and LatticeIncrementalDeterminizer, on the host, over the
// decoder's records (decoder/lattice-incremental-decoder.{h,cc} [K]; the
// reference decodes every KaldiRecognizer with
// SingleUtteranceNnet3IncrementalDecoder, src/recognizer.cc:39-43, takes
// GetLattice(NumFramesDecoded(), true) for Result / FinalResult, :678, and
// GetLattice(NumFramesInLattice(), false) + WordAlignLatticePartial for a
// PartialResult with partial words, :740-752).
//
// The GPU decoder (decoder.hip) produces the tokens and forward links of
// every frame exactly as LatticeFasterDecoder's token passing creates them
// (bit-identical to oracle.c orc_decode_kaldi).  What the incremental decoder
// adds on top of them is host-side bookkeeping, restated here:
//  - PruneActiveTokens(lattice_beam * prune_scale) before every frame whose
//    number of decoded frames is a multiple of prune_interval, with Kaldi's
//    must_prune_forward_links / must_prune_tokens flags and its delta stop
//    (a walk back stops at the first frame whose extra costs moved by no more
//    than delta: the extra costs of older frames are stale by design);
//  - UpdateLatticeDeterminization at the end of every AdvanceDecoding call:
//    once determinize_max_delay frames are undeterminized, the chunk up to
//    the frame with the fewest tokens (at least determinize_min_chunk_size
//    frames, the later frame on ties) goes to the determinizer, its last
//    frame's tokens given "fake" final costs extra_cost - tot_cost;
//  - LatticeIncrementalDeterminizer: the chunk's raw lattice (token labels on
//    arcs to the final states of the last frame's tokens; for a later chunk a
//    start state with state-labelled arcs into the re-determinized states of
//    the lattice so far, weighted by their forward costs), pruned
//    phone + word determinization (DeterminizeLatticePhonePrunedWrapper),
//    then the chunk appended to the compact lattice (arcs to token-final
//    states kept aside as final arcs, the old final costs cancelled, the
//    re-determinized states' incoming arcs re-weighted), and SetFinalCosts;
//  - FinalizeDecoding (PruneForwardLinksFinal with final costs, then every
//    frame with delta 0).
// Kaldi's decoder only ever runs these at those points, and a frame's tokens
// and links never change once created, so the host replays the schedule
// lazily (when a result is asked for) from the recorded AdvanceDecoding ends:
// the same sequence of passes on the same records.
//
// Iteration orders: tokens of a frame in the decoder's list (HashList) order,
// a token's links by graph arc.  Kaldi's PruneForwardLinks fixpoint walks
// active_toks_ (reverse creation order); where a frame's epsilon links chain
// tokens of the same frame the stale values can differ by less than delta.
// State numbering of the raw chunk and of the compact lattice is this
// restatement's own (Kaldi's depends on hash-map iteration); results depend
// on it only through exact ties.  Restated line for line by
// tests/oracle_incremental.py (parity with Kaldi itself unpinned: no Kaldi
// build or fixture here).
#pragma once
#include <set>
#include <unordered_map>
#include <vector>

#include "lattice.h"

namespace vamd {

struct IncrementalOptions {  // LatticeIncrementalDecoderConfig [K] (model.conf may override)
  float lattice_beam = 6.0f;
  int prune_interval = 25;
  float prune_scale = 0.01f;
  int determinize_max_delay = 60;
  int determinize_min_chunk_size = 20;
  long long det_max_mem = 50000000;
  int max_states = 100000;  // this build's determinization guard (Kaldi: none)
};

// One input frame: its tokens in list order and the links recorded with it
// (emitting links from the previous frame's tokens, epsilon links between
// its own), ac = the decoder's acoustic cost (cost offset included, as
// Kaldi's ForwardLink::acoustic_cost).
struct IncFrameIn {
  const int* state = nullptr;
  const float* cost = nullptr;
  int ntok = 0;
  float cost_offset = 0;  // of the emitting links into this frame
  struct Link {
    int src, dst;  // frame-local token indices (src in the previous frame if the arc emits)
    int arc;
    float ac;
    bool emit;     // the arc has a transition-id (src in the previous frame)
  };
  const Link* links = nullptr;
  int nlinks = 0;
};

// per-thread phase times in ms (add frame, prune, chunk build, determinize,
// append), accumulated for diagnostics (vamd_incremental_json reports them)
extern thread_local double vamd_inc_prof[6];

class IncrementalLattice {
 public:
  enum { kStateLabelOffset = 100000000, kTokenLabelOffset = 200000000, kMaxTokenLabel = 300000000 };

  IncrementalLattice() = default;
  void Init(const Graph* g, const std::vector<int>* tid2phone, const std::vector<char>* tid_first,
            const IncrementalOptions& opt);
  void Reset();  // InitDecoding (a new decoder segment)

  // Frame NumFramesDecoded() + 1 (frame 0 first), after Kaldi's
  // PruneActiveTokens when NumFramesDecoded() % prune_interval == 0.
  void AddFrame(const IncFrameIn& f);
  // End of an AdvanceDecoding call: UpdateLatticeDeterminization.
  void AdvanceEnd();
  void FinalizeDecoding();
  // GetLattice (lattice-incremental-decoder.cc): the compact lattice so far
  // as a WordLattice (connected, topologically sorted).  False if this
  // build's guard tripped (the caller falls back to the best path).
  bool GetLattice(int num_frames_to_include, bool use_final_probs, WordLattice* out);

  int NumFramesDecoded() const { return (int)frames_.size() - 1; }
  int NumFramesInLattice() const { return num_in_lattice_; }
  bool failed() const { return failed_; }
  bool finalized() const { return finalized_; }
  // diagnostics: chunks determinized, prune passes run
  int chunks() const { return chunks_; }
  int prune_passes() const { return prune_passes_; }

 private:
  struct HLink {
    int dst, arc;  // arc -1: excised
    float graph, ac;
    HLink() {}  // (no zero fill: a frame's arrays are written in full right after their allocation)
    HLink(int d, int a, float g, float x) : dst(d), arc(a), graph(g), ac(x) {}
  };
  struct HTok {  // 16 bytes (its index in the frame: the toks_ index - the frame's first)
    int state;
    float tot, extra;
    int frame : 31;
    bool alive : 1;
  };
  static_assert(sizeof(HTok) == 16, "token record layout");
  // A token's forward links: its emitting links (recorded with the next
  // frame) then its epsilon links, each by graph arc (emitting arcs come
  // first in the graph's per-state arc order, so this is arc order)
  struct Rng {
    int b, e;
    Rng() {}  // (as HLink)
    Rng(int b0, int e0) : b(b0), e(e0) {}
  };
  struct HFrame {
    int first = 0;          // toks_ index of the frame's first token (frame-local index 0)
    std::vector<int> toks;  // live tokens, list order
    bool must_prune_fl = true, must_prune_tok = true;
    int num_toks = -1;
    float cost_offset = 0;  // of the emitting links out of this frame (Kaldi cost_offsets_[frame])
    std::vector<HLink> emit, eps;         // links out of the frame's tokens, grouped by source
    std::vector<Rng> emit_rng, eps_rng;  // per local token: its links [b, e) (e drops as links are pruned)
  };
  template <class F> void ForLinks(int t, F&& f);  // f(HLink&) over a token's live links
  struct CArc {
    int label, next;  // final arcs: next = the source state (Kaldi's abuse of the field)
    LW w;
    std::vector<int> tids;
  };
  struct CFin {
    bool is = false;
    LW w;
    std::vector<int> tids;
  };

  float Delta() const { return opt_.lattice_beam * opt_.prune_scale; }
  void PruneForwardLinks(int f, bool* extra_costs_changed, bool* links_pruned, float delta);
  void PruneForwardLinksFinal();
  void PruneTokensForFrame(int f);
  void PruneActiveTokens(float delta);
  void ReplayDeferred();  // the deferred parts of the passes, in order (before a start-over)
  void ComputeFinalCosts(std::unordered_map<int, float>* fc, float* final_best_cost) const;
  void BuildChunk(int num_frames_to_include);  // GetLattice's chunk + AcceptRawLatticeChunk
  // LatticeIncrementalDeterminizer
  void DetInit();
  bool AcceptRawLatticeChunk(DetGraph&& raw);
  void SetFinalCosts(const std::unordered_map<int, float>* token_label2final_cost);
  int AddStateToClat();
  void AddArcToClat(int state, const CArc& arc);
  void GetNonFinalRedetStates();
  void ExportClat(WordLattice* out) const;

  const Graph* g_ = nullptr;
  const std::vector<int>* tid2phone_ = nullptr;
  const std::vector<char>* tid_first_ = nullptr;
  IncrementalOptions opt_;
  std::vector<HTok> toks_;
  std::vector<HFrame> frames_;
  std::vector<int> scratch_ce_, scratch_cp_;  // AddFrame's link counts
  struct DeferredPass {  // PruneActiveTokens' part below the next chunk
    int B;
    float delta;
    bool fl;                  // frame B's must_prune_fl at the step
    std::vector<float> extra;  // frame B + 1's tokens as the step read them
    std::vector<char> alive;
  };
  std::vector<DeferredPass> deferred_;
  bool finalized_ = false, failed_ = false;
  std::unordered_map<int, float> final_costs_;
  float final_best_cost_ = 0;
  int num_in_lattice_ = 0;
  std::unordered_map<int, int> token2label_;  // token -> label, last chunk's last frame
  int next_label_ = kTokenLabelOffset;
  int chunks_ = 0, prune_passes_ = 0;
  // determinizer state (clat_ without its final arcs)
  std::vector<std::vector<CArc>> carcs_;
  std::vector<CFin> cfin_;
  std::vector<float> fwd_;
  std::vector<std::vector<std::pair<int, int>>> arcs_in_;
  std::vector<CArc> final_arcs_;
  std::set<int> redet_;  // non-final redeterminized states (ascending)
};

}  // namespace vamd
