// Looped nnet3 planner (see nnet_plan.h).
#include "nnet_plan.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <map>
#include <set>
#include <sstream>

#include "common.h"

namespace vamd {

void BatchNormScaleOffset(const Component& c, std::vector<float>* scale,
                          std::vector<float>* offset) {
  auto mi = c.v.find("StatsMean");
  auto vi = c.v.find("StatsVar");
  if (mi == c.v.end() || vi == c.v.end()) VAMD_ERR("BatchNormComponent without statistics");
  double eps = c.f.count("Epsilon") ? c.f.at("Epsilon") : 1e-3;
  double tr = c.f.count("TargetRms") ? c.f.at("TargetRms") : 1.0;
  size_t n = mi->second.size();
  scale->resize(n);
  offset->resize(n);
  for (size_t i = 0; i < n; i++) {
    double var = std::max((double)vi->second[i], 0.0) + eps;
    double s = tr / std::sqrt(var);
    (*scale)[i] = (float)s;
    (*offset)[i] = (float)(-(double)mi->second[i] * s);
  }
}

namespace {

bool IsAffine(const std::string& t) {
  return t == "FixedAffineComponent" || t == "AffineComponent" ||
         t == "NaturalGradientAffineComponent" || t == "LinearComponent" || t == "TdnnComponent";
}
bool IsIdentity(const std::string& t) {
  return t == "NoOpComponent" || t == "GeneralDropoutComponent" || t == "DropoutComponent" ||
         t == "SpecAugmentTimeMaskComponent";
}
bool IsElementwise(const std::string& t) {
  return IsIdentity(t) || t == "RectifiedLinearComponent" || t == "BatchNormComponent" ||
         t == "ScaleAndOffsetComponent";
}

// A by-name reference used while building (resolved to stored nodes later).
struct NRef {
  std::string node;
  int offset = 0, col = 0;
};

struct TmpSeg { NRef ref; int col0, dim; };
struct TmpInstr { int op; NRef ref; float c = 0.f; };
struct TmpPart { int col0, dim; std::vector<TmpInstr> prog; };
struct TmpStage { EpiStage st; NRef ref; };
struct TmpOp {
  int kind;
  std::string name;
  bool llh = false;
  int N = 0, K = 0, weight = -1;
  std::vector<TmpSeg> segs;
  std::vector<TmpPart> parts;
  std::vector<TmpStage> epi;
};

struct Builder {
  const Nnet& nn;
  float acoustic_scale;
  NnetPlan plan;
  std::vector<TmpOp> ops;
  std::map<std::string, int> consumers;
  std::map<std::string, int> op_of;  // component node -> op that produced its value
  std::set<std::string> stored;      // node names that must be materialised
  int tmp_counter = 0;

  Builder(const Nnet& n, float ac) : nn(n), acoustic_scale(ac) {}

  void CountRefs(const Desc& d, int mult) {
    if (d.kind == Desc::NODE) { consumers[d.node] += mult; return; }
    for (auto& a : d.args) CountRefs(a, mult);
  }

  void Deps(const Desc& d, std::vector<std::string>* out) {
    if (d.kind == Desc::NODE) { out->push_back(d.node); return; }
    for (auto& a : d.args) Deps(a, out);
  }

  // topological order of the nodes needed for `root`
  void Topo(const std::string& n, std::set<std::string>* seen, std::vector<std::string>* order) {
    if (seen->count(n)) return;
    seen->insert(n);
    const NnetNode& nd = nn.Node(n);
    std::vector<std::string> deps;
    if (nd.kind == NnetNode::COMPONENT || nd.kind == NnetNode::OUTPUT) Deps(nd.input, &deps);
    if (nd.kind == NnetNode::DIM_RANGE) deps.push_back(nd.src);
    for (auto& d : deps) Topo(d, seen, order);
    order->push_back(n);
  }

  // Resolve a reference to a node value usable from device memory.
  NRef Resolve(const std::string& name, int offset) {
    const NnetNode& nd = nn.Node(name);
    if (nd.kind == NnetNode::DIM_RANGE) {
      NRef r = Resolve(nd.src, offset);
      r.col += nd.dim_offset;
      return r;
    }
    if (nd.kind == NnetNode::INPUT) {
      if (name != "input")
        VAMD_ERR("nnet input node '" << name << "' is not supported yet (i-vector input: "
                                        "see DESIGN.md, next rows)");
    } else if (nd.kind == NnetNode::COMPONENT) {
      auto it = op_of.find(name);
      if (it == op_of.end() || ops[it->second].name != name)
        VAMD_ERR("internal: value of node " << name << " is not materialisable");
    } else {
      VAMD_ERR("cannot reference output node " << name);
    }
    stored.insert(name);
    NRef r;
    r.node = name;
    r.offset = offset;
    return r;
  }

  // Plain node reference with time offset (and optional scale).
  bool SimpleRef(const Desc& d, std::string* node, int* off, float* scale, bool* scaled) {
    if (d.kind == Desc::NODE) { *node = d.node; return true; }
    if (d.kind == Desc::OFFSET) {
      if (!SimpleRef(d.args[0], node, off, scale, scaled)) return false;
      *off += d.t;
      return true;
    }
    if (d.kind == Desc::SCALE && scale) {
      if (*scaled) return false;
      *scaled = true;
      *scale = d.scale;
      return SimpleRef(d.args[0], node, off, scale, scaled);
    }
    if (d.kind == Desc::IFDEFINED) return SimpleRef(d.args[0], node, off, scale, scaled);
    return false;
  }

  void Compile(const Desc& d, int toff, std::vector<TmpInstr>* prog) {
    switch (d.kind) {
      case Desc::NODE: {
        TmpInstr in{GInstr::PUSH, Resolve(d.node, toff)};
        prog->push_back(in);
        break;
      }
      case Desc::OFFSET: Compile(d.args[0], toff + d.t, prog); break;
      case Desc::IFDEFINED: Compile(d.args[0], toff, prog); break;
      case Desc::SCALE: {
        Compile(d.args[0], toff, prog);
        TmpInstr in{GInstr::SCALE, NRef(), d.scale};
        prog->push_back(in);
        break;
      }
      case Desc::SUM: {
        Compile(d.args[0], toff, prog);
        for (size_t i = 1; i < d.args.size(); i++) {
          Compile(d.args[i], toff, prog);
          TmpInstr in{GInstr::ADD, NRef()};
          prog->push_back(in);
        }
        break;
      }
      case Desc::CONST: {
        TmpInstr in{GInstr::CONST, NRef(), d.scale};
        prog->push_back(in);
        break;
      }
      case Desc::REPLACE_INDEX: {
        // ReplaceIndex(ivector, t, 0): the chunk's i-vector (Kaldi's looped
        // decodable supplies one i-vector row per chunk)
        const Desc& in = d.args[0];
        if (in.kind != Desc::NODE || !nn.HasNode(in.node) ||
            nn.Node(in.node).kind != NnetNode::INPUT || in.node == "input" || d.t != 0)
          VAMD_ERR("ReplaceIndex is supported only as ReplaceIndex(<ivector input>, t, 0)");
        stored.insert(in.node);
        TmpInstr instr{GInstr::PUSH_JOB, NRef()};
        instr.ref.node = in.node;
        prog->push_back(instr);
        break;
      }
      default:
        VAMD_ERR("descriptor kind " << (int)d.kind << " unsupported in a gather (Round: next rows)");
    }
  }

  // New GATHER op evaluating descriptor d; returns op index.
  int MakeGather(const Desc& d, const std::string& name) {
    TmpOp op;
    op.kind = Op::GATHER;
    op.name = name;
    std::vector<const Desc*> parts;
    if (d.kind == Desc::APPEND) for (auto& a : d.args) parts.push_back(&a);
    else parts.push_back(&d);
    int col = 0;
    for (const Desc* p : parts) {
      TmpPart tp;
      tp.col0 = col;
      tp.dim = nn.DescDim(*p);
      Compile(*p, 0, &tp.prog);
      col += tp.dim;
      op.parts.push_back(std::move(tp));
    }
    op.N = col;
    ops.push_back(std::move(op));
    int idx = (int)ops.size() - 1;
    op_of[name] = idx;
    return idx;
  }

  int AddVec(std::vector<float> v, int dim) {
    if ((int)v.size() != dim) {  // block-dim tiling (BatchNorm block_dim < dim)
      if (v.empty() || dim % (int)v.size()) VAMD_ERR("bad per-dim vector size");
      std::vector<float> t(dim);
      for (int i = 0; i < dim; i++) t[i] = v[i % v.size()];
      v.swap(t);
    }
    plan.vecs.push_back(std::move(v));
    return (int)plan.vecs.size() - 1;
  }

  void AppendComponentStage(TmpOp& op, const Component& c) {
    int dim = op.N;
    if (c.type == "RectifiedLinearComponent") {
      TmpStage s;
      s.st.kind = EpiStage::RELU;
      op.epi.push_back(s);
    } else if (c.type == "BatchNormComponent") {
      bool test_mode = c.b.count("TestMode") ? c.b.at("TestMode") : false;
      if (!test_mode)
        VAMD_LOG("BatchNormComponent not in test mode; using stored stats (SetBatchnormTestMode)");
      std::vector<float> s, o;
      BatchNormScaleOffset(c, &s, &o);
      TmpStage st;
      st.st.kind = EpiStage::MUL_ADD;
      st.st.vec0 = AddVec(s, dim);
      st.st.vec1 = AddVec(o, dim);
      op.epi.push_back(st);
    } else if (c.type == "ScaleAndOffsetComponent") {
      TmpStage st;
      st.st.kind = EpiStage::MUL_ADD;
      st.st.vec0 = AddVec(c.v.at("Scales"), dim);
      st.st.vec1 = AddVec(c.v.at("Offsets"), dim);
      op.epi.push_back(st);
    } else if (!IsIdentity(c.type)) {
      VAMD_ERR("unsupported element-wise component " << c.type);
    }
  }

  // Try to fuse element-wise node input `d` into the op producing its single
  // plain-node leaf.  Fills adds (leaf-to-root order).  Returns op or -1.
  int FindFusable(const Desc& d, std::vector<TmpStage>* adds) {
    if (d.kind == Desc::NODE) {
      const NnetNode& nd = nn.Node(d.node);
      if (nd.kind != NnetNode::COMPONENT) return -1;
      auto it = op_of.find(d.node);
      if (it == op_of.end() || ops[it->second].name != d.node) return -1;
      if (consumers[d.node] != 1) return -1;
      return it->second;
    }
    if (d.kind != Desc::SUM) return -1;
    for (size_t k = 0; k < d.args.size() && k < 2; k++) {
      std::vector<TmpStage> inner;
      int o = FindFusable(d.args[k], &inner);
      if (o < 0) continue;
      std::vector<TmpStage> mine = inner;
      bool ok = true;
      for (size_t j = 0; j < d.args.size(); j++) {
        if (j == k) continue;
        std::string n;
        int off = 0;
        float sc = 1.f;
        bool scaled = false;
        if (!SimpleRef(d.args[j], &n, &off, &sc, &scaled)) { ok = false; break; }
        TmpStage st;
        st.st.kind = EpiStage::ADD_NODE;
        st.st.c = sc;
        st.st.scaled = scaled;
        st.ref = Resolve(n, off);
        mine.push_back(st);
      }
      if (!ok) return -1;
      *adds = mine;
      return o;
    }
    return -1;
  }

  void Build(int fpc, int fss) {
    if (!nn.HasNode("output")) VAMD_ERR("nnet has no 'output' node");
    std::set<std::string> seen;
    std::vector<std::string> order;
    Topo("output", &seen, &order);
    for (auto& n : order) {
      const NnetNode& nd = nn.Node(n);
      if (nd.kind == NnetNode::DIM_RANGE) consumers[nd.src] += 2;  // forces storage
      if (nd.kind == NnetNode::COMPONENT) {
        const Component& c = nn.components.at(nd.component);
        int mult = c.type == "TdnnComponent" ? std::max<int>(2, c.time_offsets.size()) : 1;
        CountRefs(nd.input, mult);
      } else if (nd.kind == NnetNode::OUTPUT) {
        CountRefs(nd.input, 1);
      }
    }
    for (auto& n : order) {
      const NnetNode& nd = nn.Node(n);
      if (nd.kind == NnetNode::INPUT || nd.kind == NnetNode::DIM_RANGE) continue;
      if (nd.kind == NnetNode::OUTPUT) {
        if (nd.input.kind != Desc::NODE) VAMD_ERR("output node descriptor must be a plain node");
        const std::string& y = nd.input.node;
        auto it = op_of.find(y);
        if (it == op_of.end() || ops[it->second].name != y || consumers[y] != 1)
          VAMD_ERR("nnet output " << y << " is also consumed elsewhere (unsupported)");
        TmpOp& op = ops[it->second];
        op.llh = true;
        TmpStage st;
        st.st.kind = EpiStage::SCALE;
        st.st.c = acoustic_scale;
        op.epi.push_back(st);
        continue;
      }
      auto cit = nn.components.find(nd.component);
      if (cit == nn.components.end()) VAMD_ERR("missing component " << nd.component);
      const Component& c = cit->second;
      if (IsAffine(c.type)) {
        TmpOp op;
        op.kind = Op::GEMM;
        op.name = n;
        const Matrix* W = c.m.count("LinearParams") ? &c.m.at("LinearParams") : nullptr;
        if (!W && c.m.count("Params")) W = &c.m.at("Params");
        if (!W) VAMD_ERR("affine component " << nd.component << " without parameters");
        std::vector<const Desc*> parts;
        if (nd.input.kind == Desc::APPEND) for (auto& a : nd.input.args) parts.push_back(&a);
        else parts.push_back(&nd.input);
        // simple (node, offset) parts; anything else is materialised first
        std::vector<NRef> prefs;
        std::vector<int> pdims;
        for (const Desc* p : parts) {
          std::string nm;
          int off = 0;
          bool scaled = false;
          if (SimpleRef(*p, &nm, &off, nullptr, &scaled)) {
            prefs.push_back(Resolve(nm, off));
          } else {
            std::string tmp = n + ".input" + std::to_string(tmp_counter++);
            MakeGather(*p, tmp);
            prefs.push_back(Resolve(tmp, 0));
          }
          pdims.push_back(nn.DescDim(*p));
        }
        std::vector<int> toffs = c.type == "TdnnComponent" ? c.time_offsets : std::vector<int>{0};
        if (toffs.empty()) VAMD_ERR("TdnnComponent without time offsets");
        int col = 0;
        for (int to : toffs)
          for (size_t j = 0; j < prefs.size(); j++) {
            TmpSeg s;
            s.ref = prefs[j];
            s.ref.offset += to;
            s.col0 = col;
            s.dim = pdims[j];
            col += pdims[j];
            op.segs.push_back(s);
          }
        if (col != W->cols)
          VAMD_ERR("component " << nd.component << ": input dim " << col << " != weight cols "
                                << W->cols);
        op.K = col;
        op.N = W->rows;
        plan.mats.push_back(*W);
        op.weight = (int)plan.mats.size() - 1;
        auto b = c.v.find("BiasParams");
        if (b != c.v.end() && !b->second.empty()) {
          TmpStage st;
          st.st.kind = EpiStage::BIAS;
          st.st.vec0 = AddVec(b->second, op.N);
          op.epi.push_back(st);
        }
        ops.push_back(std::move(op));
        op_of[n] = (int)ops.size() - 1;
      } else if (IsElementwise(c.type)) {
        std::vector<TmpStage> adds;
        int o = FindFusable(nd.input, &adds);
        if (o < 0) o = MakeGather(nd.input, n);
        TmpOp& op = ops[o];
        for (auto& a : adds) op.epi.push_back(a);
        AppendComponentStage(op, c);
        op.name = n;
        op_of[n] = o;
      } else {
        VAMD_ERR("unsupported nnet3 component type " << c.type);
      }
    }
    Finish(fpc, fss);
  }

  void Finish(int fpc, int fss) {
    // stored nodes
    std::map<std::string, int> sidx;
    auto get_stored = [&](const std::string& name) {
      auto it = sidx.find(name);
      if (it != sidx.end()) return it->second;
      StoredNode s;
      s.name = name;
      s.dim = nn.HasNode(name) ? nn.OutputDimOf(name) : -1;
      const bool in = nn.HasNode(name) && nn.Node(name).kind == NnetNode::INPUT;
      s.is_input = in && name == "input";
      s.is_ivector = in && name != "input";
      if (s.dim < 0) {  // temporary gather node
        for (auto& o : ops) if (o.name == name) s.dim = o.N;
      }
      plan.nodes.push_back(s);
      int i = (int)plan.nodes.size() - 1;
      sidx[name] = i;
      if (s.is_input) { plan.input_node = i; plan.input_dim = s.dim; }
      if (s.is_ivector) {
        if (plan.ivector_node >= 0) VAMD_ERR("more than one per-chunk nnet input");
        plan.ivector_node = i;
        plan.ivector_dim = s.dim;
      }
      return i;
    };
    get_stored("input");
    for (auto& n : stored) get_stored(n);
    std::map<int, int> producer;  // stored node -> op
    int llh_op = -1;
    for (size_t i = 0; i < ops.size(); i++) {
      if (ops[i].llh) { llh_op = (int)i; continue; }
      auto it = sidx.find(ops[i].name);
      if (it == sidx.end()) continue;  // output consumed only via fusion?  dead
      producer[it->second] = (int)i;
    }
    if (llh_op < 0) VAMD_ERR("no op produces the nnet output");
    // convert
    std::vector<Op> conv(ops.size());
    std::vector<bool> live(ops.size(), false);
    for (size_t i = 0; i < ops.size(); i++) {
      const TmpOp& t = ops[i];
      Op& o = conv[i];
      o.kind = t.kind;
      o.name = t.name;
      o.N = t.N;
      o.K = t.K;
      o.weight = t.weight;
      o.out_node = t.llh ? -1 : (sidx.count(t.name) ? sidx[t.name] : -2);
      live[i] = o.out_node != -2;
      std::set<int> deps;
      auto dep = [&](int node) {
        if (node == plan.input_node) return;
        deps.insert(producer.at(node));
      };
      for (auto& s : t.segs) {
        ASegment a{sidx.at(s.ref.node), s.ref.offset, s.col0, s.dim, s.ref.col};
        dep(a.node);
        o.segs.push_back(a);
      }
      for (auto& p : t.parts) {
        GPart gp{p.col0, p.dim, {}};
        for (auto& in : p.prog) {
          GInstr g;
          g.op = in.op;
          g.c = in.c;
          if (in.op == GInstr::PUSH) {
            g.node = sidx.at(in.ref.node);
            g.offset = in.ref.offset;
            g.src_col = in.ref.col;
            dep(g.node);
          } else if (in.op == GInstr::PUSH_JOB) {
            g.node = sidx.at(in.ref.node);  // no time dependency, no producer
          }
          gp.prog.push_back(g);
        }
        o.parts.push_back(gp);
      }
      for (auto& s : t.epi) {
        EpiStage e = s.st;
        if (e.kind == EpiStage::ADD_NODE) {
          e.node = sidx.at(s.ref.node);
          e.offset = s.ref.offset;
          e.src_col = s.ref.col;
          dep(e.node);
        }
        o.epi.push_back(e);
      }
      o.deps.assign(deps.begin(), deps.end());
    }
    // topological sort of live ops (Kahn, stable by creation order)
    std::vector<int> order;
    std::vector<int> state(ops.size(), 0);
    std::function<void(int)> visit = [&](int i) {
      if (state[i] == 2) return;
      if (state[i] == 1) VAMD_ERR("cycle in fused nnet op graph");
      state[i] = 1;
      for (int d : conv[i].deps) visit(d);
      state[i] = 2;
      order.push_back(i);
    };
    for (size_t i = 0; i < ops.size(); i++)
      if (live[i]) visit((int)i);
    std::map<int, int> remap;
    for (size_t k = 0; k < order.size(); k++) remap[order[k]] = (int)k;
    for (int i : order) {
      Op o = conv[i];
      for (auto& d : o.deps) d = remap.at(d);
      plan.ops.push_back(o);
    }
    for (auto& [node, op] : producer) producer[node] = remap.count(op) ? remap[op] : -1;
    int llh = remap.at(llh_op);
    plan.out_dim = plan.ops[llh].N;
    Schedule(fpc, fss, llh, producer);
  }

  // refs of an op: (stored node, time offset)
  static std::vector<std::pair<int, int>> Refs(const Op& o) {
    std::vector<std::pair<int, int>> r;
    for (auto& s : o.segs) r.push_back({s.node, s.offset});
    for (auto& p : o.parts)
      for (auto& g : p.prog)
        if (g.op == GInstr::PUSH) r.push_back({g.node, g.offset});
    for (auto& e : o.epi)
      if (e.kind == EpiStage::ADD_NODE) r.push_back({e.node, e.offset});
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
    return r;
  }

  // needed times per op for the given output times
  std::vector<std::set<int>> Needed(const std::set<int>& out_times, int llh,
                                    const std::map<int, int>& producer, std::set<int>* input_times) {
    std::vector<std::set<int>> need(plan.ops.size());
    need[llh] = out_times;
    for (int o = (int)plan.ops.size() - 1; o >= 0; o--) {
      auto refs = Refs(plan.ops[o]);
      for (int t : need[o])
        for (auto& [m, off] : refs) {
          if (m == plan.input_node) input_times->insert(t + off);
          else need[producer.at(m)].insert(t + off);
        }
    }
    return need;
  }

  void Schedule(int fpc, int fss, int llh, const std::map<int, int>& producer) {
    if (fss < 1) VAMD_ERR("bad frame_subsampling_factor " << fss);
    if (fpc < fss) fpc = fss;
    if (fpc % fss) fpc += fss - fpc % fss;  // GetChunkSize rounding [K]
    plan.fpc = fpc;
    plan.fss = fss;
    plan.opc = fpc / fss;
    size_t nops = plan.ops.size();
    // Kaldi ComputeSimpleNnetContext (modulus 1): context of the output at t=0
    {
      std::set<int> in;
      Needed({0}, llh, producer, &in);
      plan.left_context = std::max(0, -*in.begin());
      plan.right_context = std::max(0, *in.rbegin());
    }
    int span = plan.left_context + plan.right_context + fpc;
    int C = span / fpc + 3;
    std::vector<std::vector<std::set<int>>> need(C + 1);
    for (int c = 0; c <= C; c++) {
      std::set<int> out;
      for (int i = 0; i < plan.opc; i++) out.insert(c * fpc + fss * i);
      std::set<int> in;
      need[c] = Needed(out, llh, producer, &in);
    }
    for (size_t o = 0; o < nops; o++) {
      auto newset = [&](int c) {
        std::vector<int> p;
        for (int t : need[c][o]) {
          bool old = false;
          for (int cc = 0; cc < c && !old; cc++) old = need[cc][o].count(t) != 0;
          if (!old) p.push_back(t - c * fpc);
        }
        return p;
      };
      std::vector<int> a = newset(C), b = newset(C - 1);
      if (a != b) VAMD_ERR("nnet op " << plan.ops[o].name << " is not periodic at frames_per_chunk "
                                      << fpc);
      plan.ops[o].pattern = a;
    }
    // priming: smallest P such that every needed value is computed correctly
    const int max_p = span / fpc + 4;
    for (int P = 0; P <= max_p; P++) {
      std::vector<std::set<int>> correct(plan.nodes.size());
      bool ok = true;
      int max_age = 0;
      std::vector<int> latest(plan.nodes.size(), INT32_MIN);
      for (int c = -P; c <= C && ok; c++) {
        for (size_t o = 0; o < nops; o++) {
          const Op& op = plan.ops[o];
          auto refs = Refs(op);
          for (int k : op.pattern) {
            int t = k + c * fpc;
            bool good = true;
            for (auto& [m, off] : refs) {
              if (m == plan.input_node) continue;
              if (!correct[m].count(t + off)) { good = false; break; }
              max_age = std::max(max_age, latest[m] - (t + off));
            }
            if (good && op.out_node >= 0) correct[op.out_node].insert(t);
            if (op.out_node >= 0) latest[op.out_node] = std::max(latest[op.out_node], t);
            if (!good && op.out_node < 0 && c >= 0) ok = false;
          }
        }
        if (c >= 0 && ok) {
          for (size_t o = 0; o < nops && ok; o++) {
            if (plan.ops[o].out_node < 0) continue;
            for (int t : need[std::min(c, C)][o])
              if (!correct[plan.ops[o].out_node].count(t)) { ok = false; break; }
          }
        }
      }
      if (ok) {
        plan.priming_chunks = P;
        plan.max_age = max_age;
        break;
      }
      if (P == max_p) VAMD_ERR("could not find a priming schedule for the nnet");
    }
    plan.flops_per_chunk = 0;
    for (auto& o : plan.ops)
      if (o.kind == Op::GEMM) plan.flops_per_chunk += 2.0 * o.pattern.size() * o.N * (double)o.K;
  }
};

}  // namespace

int NnetPlan::RingFrames(int jobs_per_slot) const {
  int need = max_age + jobs_per_slot * fpc + fpc + 8;
  int r = 64;
  while (r < need) r <<= 1;
  return r;
}

std::string NnetPlan::Describe() const {
  std::ostringstream os;
  os << "nnet plan: fpc=" << fpc << " fss=" << fss << " L=" << left_context
     << " R=" << right_context << " priming=" << priming_chunks << " max_age=" << max_age
     << " ops=" << ops.size() << " stored=" << nodes.size()
     << " MFLOP/chunk=" << flops_per_chunk * 1e-6 << "\n";
  for (auto& o : ops) {
    os << "  " << (o.kind == Op::GEMM ? "GEMM  " : "GATHER") << " " << o.name << " N=" << o.N
       << " K=" << o.K << " rows/chunk=" << o.pattern.size() << " -> "
       << (o.out_node < 0 ? std::string("LLH") : nodes[o.out_node].name) << " epi=";
    for (auto& e : o.epi) os << e.kind;
    os << "\n";
  }
  return os.str();
}

NnetPlan BuildNnetPlan(const Nnet& nnet, int frames_per_chunk, int fss, float acoustic_scale) {
  Builder b(nnet, acoustic_scale);
  b.Build(frames_per_chunk, fss);
  return std::move(b.plan);
}

}  // namespace vamd
