// Static decode graphs for lookahead models and runtime grammars (SURVEY.md
// §8f-2).
//
// Models like vosk-model-small-en-us ship no HCLG: the reference composes
// HCLr.fst (olabel_lookahead; H∘C∘L with output labels relabeled for label
// lookahead) with Gr.fst (ngram) on the fly, `LookaheadComposeFst(*hcl_fst_,
// *g_fst_, disambig_)` (src/recognizer.cc:31-37), and the grammar recognizer
// composes HCLr with a bigram estimated from the phrase list
// (src/recognizer.cc:49-108, src/language_model.cc).  The GPU decoder walks a
// CSR graph in HBM, so the composition is expanded once on the host into a
// static graph with the states and arcs of the reference's lazy one.
// ComposeFst with an olabel_lookahead first FST runs OpenFST's default
// MATCH_OUTPUT lookahead filter chain [O: compose.h CreateBase,
// lookahead-filter.h], restated in graph_compose.cc:
//
//  * alternative sequence filter: the grammar's epsilon (backoff) arcs are
//    taken before HCLr's output-epsilon arcs, never after them within a word;
//  * label lookahead: an HCLr output-epsilon move is expanded only if some
//    output label reachable from its destination is on an arc of the grammar
//    state (or a final state is reachable and the grammar state is final);
//    reachable label sets per strongly connected component of HCLr's
//    output-epsilon subgraph, as sorted interval lists;
//  * weight pushing: such a move carries the log-sum of the reachable grammar
//    arcs' weights (FastLogAccumulator) minus the weight pushed so far, which
//    the state keeps quantized to 1/1024; word and backoff arcs subtract it;
//  * label pushing: when exactly one grammar arc is reachable (and no final),
//    that arc is taken on the move itself (its word output early, the grammar
//    state advanced), and the state keeps the label HCLr must still output;
//  * disambiguation transition-ids (disambig_tid.int) become epsilon;
//  * the result is trimmed (states that reach no final state removed) and
//    renumbered in breadth-first order from the start state over each
//    state's emitting arcs then epsilon arcs (the canonical order
//    tests/oracle_graph.py reproduces).
//
// Not reproduced: the composed state numbering (OpenFST numbers states as
// the decoder first visits them; Kaldi's HashList order depends on it) and
// the exact interval count of the final label in OpenFST's reachability data
// (it only selects between two summation orders of the lookahead weight).
#pragma once
#include <string>
#include <vector>

#include "model_io.h"

namespace vamd {

void ComposeLookahead(const HostFst& hcl, const HostFst& g, const std::vector<int>& disambig,
                      HostFst* out);

// LanguageModelEstimator (src/language_model.cc:27-211) with the grammar
// recognizer's options (order 2, discount 0.5, src/recognizer.cc:68-71):
// counts of every n-gram of each sentence plus the end-of-sentence event,
// parents accumulate their descendants' counts, each active history becomes
// one state with arcs -log(count * discount / total) and a backoff arc
// -log(1 - discount), ilabel-sorted.
void EstimateGrammarLm(const std::vector<std::vector<int>>& sentences, int order, float discount,
                       HostFst* out);

// The grammar recognizer's phrase list: a JSON array of strings
// (src/recognizer.cc:60-92).  Words are split on ' ' and looked up in the
// word table; unknown words are dropped with a warning.  Throws if the text
// is not an array of strings.
std::vector<std::vector<int>> ParseGrammarJson(const std::string& json, const SymbolTable& words);

}  // namespace vamd
