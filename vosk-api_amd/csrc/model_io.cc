// Model-format readers (see model_io.h for the reference call sites).
#include "model_io.h"

#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <iterator>
#include <limits>
#include <cstring>
#include <fstream>
#include <iostream>
#include <mutex>

#include "common.h"

namespace vamd {

// ---------------------------------------------------------------------------
// logging (format of the reference's handler: src/model.cc:34-104)
// ---------------------------------------------------------------------------
static std::atomic<int> g_log_level{0};
int LogLevel() { return g_log_level.load(); }
void SetLogLevel(int l) { g_log_level.store(l); }
void LogMessage(const char* kind, const std::string& msg) {
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  std::cerr << kind << " (VoskAPI:amd) " << msg << "\n";
}

bool FileExists(const std::string& path) {
  struct stat b;
  return stat(path.c_str(), &b) == 0;
}

static std::string Trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

std::map<std::string, std::string> ReadConfigFile(const std::string& path) {
  std::ifstream in(path);
  if (!in) VAMD_ERR("cannot open config file " << path);
  std::map<std::string, std::string> kv;
  std::string ln;
  while (std::getline(in, ln)) {
    size_t h = ln.find('#');
    if (h != std::string::npos) ln = ln.substr(0, h);
    ln = Trim(ln);
    if (ln.rfind("--", 0) != 0) continue;
    size_t eq = ln.find('=');
    if (eq == std::string::npos) kv[ln.substr(2)] = "true";
    else kv[Trim(ln.substr(2, eq - 2))] = Trim(ln.substr(eq + 1));
  }
  return kv;
}

static bool ParseBool(const std::string& v) { return v == "true" || v == "1" || v == "T"; }

void MfccOptions::Apply(const std::map<std::string, std::string>& kv) {
  for (auto& [k, v] : kv) {
    if (k == "sample-frequency") samp_freq = std::stof(v);
    else if (k == "frame-shift") frame_shift_ms = std::stof(v);
    else if (k == "frame-length") frame_length_ms = std::stof(v);
    else if (k == "dither") dither = std::stof(v);
    else if (k == "preemphasis-coefficient") preemph_coeff = std::stof(v);
    else if (k == "remove-dc-offset") remove_dc_offset = ParseBool(v);
    else if (k == "window-type") window_type = v;
    else if (k == "round-to-power-of-two") round_to_power_of_two = ParseBool(v);
    else if (k == "blackman-coeff") blackman_coeff = std::stof(v);
    else if (k == "snip-edges") snip_edges = ParseBool(v);
    else if (k == "num-mel-bins") num_bins = std::stoi(v);
    else if (k == "num-ceps") num_ceps = std::stoi(v);
    else if (k == "use-energy") use_energy = ParseBool(v);
    else if (k == "raw-energy") raw_energy = ParseBool(v);
    else if (k == "htk-compat") htk_compat = ParseBool(v);
    else if (k == "energy-floor") energy_floor = std::stof(v);
    else if (k == "low-freq") low_freq = std::stof(v);
    else if (k == "high-freq") high_freq = std::stof(v);
    else if (k == "cepstral-lifter") cepstral_lifter = std::stof(v);
    else if (k == "allow-downsample") allow_downsample = ParseBool(v);
    else if (k == "allow-upsample") allow_upsample = ParseBool(v);
    else if (k == "use-log-fbank") use_log_fbank = ParseBool(v);
    else if (k == "use-power") use_power = ParseBool(v);
    else VAMD_WARN("ignoring unsupported feature option --" << k);
  }
}

static std::vector<int> ParseColonList(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ':'))
    if (!Trim(tok).empty()) out.push_back(std::stoi(tok));
  return out;
}

void ApplyModelOptions(const std::map<std::string, std::string>& kv, DecoderOptions* dec,
                       DecodableOptions* dcb, EndpointConfig* ep) {
  for (auto& [k, v] : kv) {
    if (k == "beam") dec->beam = std::stof(v);
    else if (k == "max-active") dec->max_active = std::stoi(v);
    else if (k == "min-active") dec->min_active = std::stoi(v);
    else if (k == "lattice-beam") dec->lattice_beam = std::stof(v);
    else if (k == "prune-interval") dec->prune_interval = std::stoi(v);
    else if (k == "beam-delta") dec->beam_delta = std::stof(v);
    else if (k == "hash-ratio") dec->hash_ratio = std::stof(v);
    else if (k == "determinize-max-delay") dec->determinize_max_delay = std::stoi(v);
    else if (k == "determinize-min-chunk-size") dec->determinize_min_chunk_size = std::stoi(v);
    else if (k == "determinize-max-active") {}  // (not read by UpdateLatticeDeterminization)
    else if (k == "acoustic-scale") dcb->acoustic_scale = std::stof(v);
    else if (k == "frame-subsampling-factor") dcb->frame_subsampling_factor = std::stoi(v);
    else if (k == "frames-per-chunk") dcb->frames_per_chunk = std::stoi(v);
    else if (k == "extra-left-context-initial") dcb->extra_left_context_initial = std::stoi(v);
    else if (k == "endpoint.silence-phones") ep->silence_phones = ParseColonList(v);
    else if (k.rfind("endpoint.rule", 0) == 0 && k.size() > 15) {
      int r = k[13] - '1';
      if (r < 0 || r > 4) VAMD_ERR("bad endpoint rule option " << k);
      std::string f = k.substr(15);
      if (f == "must-contain-nonsilence") ep->rule[r].must_contain_nonsilence = ParseBool(v);
      else if (f == "min-trailing-silence") ep->rule[r].min_trailing_silence = std::stof(v);
      else if (f == "max-relative-cost") ep->rule[r].max_relative_cost = std::stof(v);
      else if (f == "min-utterance-length") ep->rule[r].min_utterance_length = std::stof(v);
      else VAMD_WARN("ignoring option --" << k);
    } else {
      VAMD_WARN("ignoring unsupported model option --" << k);
    }
  }
}

// ---------------------------------------------------------------------------
// Kaldi binary reader
// ---------------------------------------------------------------------------
namespace {
struct KReader {
  const std::string& d;
  size_t p;
  explicit KReader(const std::string& data) : d(data), p(0) {
    if (d.size() < 2 || d[0] != '\0' || d[1] != 'B') VAMD_ERR("not a binary Kaldi file");
    p = 2;
  }
  void Need(size_t n) const {
    if (p + n > d.size()) VAMD_ERR("unexpected end of Kaldi file at " << p);
  }
  void SkipWs() {
    while (p < d.size() && (d[p] == ' ' || d[p] == '\t' || d[p] == '\n' || d[p] == '\r')) ++p;
  }
  std::string Token() {
    SkipWs();
    size_t e = p;
    while (e < d.size() && d[e] != ' ' && d[e] != '\t' && d[e] != '\n' && d[e] != '\r') ++e;
    std::string t = d.substr(p, e - p);
    p = e;
    if (p < d.size() && d[p] == ' ') ++p;
    return t;
  }
  std::string PeekToken() {
    size_t save = p;
    std::string t = Token();
    p = save;
    return t;
  }
  void Expect(const std::string& t) {
    std::string g = Token();
    if (g != t) VAMD_ERR("expected token " << t << " got '" << g << "' at " << p);
  }
  int32_t I32() {
    Need(5);
    if (d[p] != 4) VAMD_ERR("bad int32 size byte at " << p);
    int32_t v;
    memcpy(&v, d.data() + p + 1, 4);
    p += 5;
    return v;
  }
  float F32() {
    Need(1);
    if (d[p] == 4) {
      Need(5);
      float v;
      memcpy(&v, d.data() + p + 1, 4);
      p += 5;
      return v;
    }
    if (d[p] == 8) {
      Need(9);
      double v;
      memcpy(&v, d.data() + p + 1, 8);
      p += 9;
      return (float)v;
    }
    VAMD_ERR("bad float size byte at " << p);
  }
  bool Bool() {
    SkipWs();
    Need(1);
    char c = d[p++];
    if (c != 'T' && c != 'F') VAMD_ERR("bad bool at " << p);
    return c == 'T';
  }
  std::vector<int> IntVector() {
    Need(5);
    int sz = d[p];
    int32_t n;
    memcpy(&n, d.data() + p + 1, 4);
    p += 5;
    if (n < 0 || (sz != 4 && sz != 8 && sz != 2 && sz != 1)) VAMD_ERR("bad int vector");
    Need((size_t)n * sz);
    std::vector<int> v(n);
    for (int i = 0; i < n; i++) {
      int64_t x = 0;
      if (sz == 4) { int32_t y; memcpy(&y, d.data() + p, 4); x = y; }
      else if (sz == 8) { memcpy(&x, d.data() + p, 8); }
      else if (sz == 2) { int16_t y; memcpy(&y, d.data() + p, 2); x = y; }
      else { x = (int8_t)d[p]; }
      v[i] = (int)x;
      p += sz;
    }
    return v;
  }
  std::vector<float> Vector() {
    std::string t = Token();
    int n = I32();
    std::vector<float> v(n);
    if (t == "FV") {
      Need((size_t)n * 4);
      memcpy(v.data(), d.data() + p, (size_t)n * 4);
      p += (size_t)n * 4;
    } else if (t == "DV") {
      Need((size_t)n * 8);
      for (int i = 0; i < n; i++) { double x; memcpy(&x, d.data() + p, 8); v[i] = (float)x; p += 8; }
    } else {
      VAMD_ERR("unsupported vector type " << t);
    }
    return v;
  }
  Matrix Mat() {
    std::string t = Token();
    Matrix m;
    m.rows = I32();
    m.cols = I32();
    size_t n = (size_t)m.rows * m.cols;
    m.data.resize(n);
    if (t == "FM") {
      Need(n * 4);
      memcpy(m.data.data(), d.data() + p, n * 4);
      p += n * 4;
    } else if (t == "DM") {
      Need(n * 8);
      for (size_t i = 0; i < n; i++) { double x; memcpy(&x, d.data() + p, 8); m.data[i] = (float)x; p += 8; }
    } else {
      VAMD_ERR("unsupported matrix type " << t << " (compressed matrices are not supported)");
    }
    return m;
  }
  double F64() {
    Need(1);
    if (d[p] == 8) {
      Need(9);
      double v;
      memcpy(&v, d.data() + p + 1, 8);
      p += 9;
      return v;
    }
    return F32();
  }
  // double-precision matrix / vector / packed symmetric matrix (DM/FM, DV/FV, DP/FP)
  std::vector<double> Mat64(int* rows, int* cols) {
    std::string t = Token();
    *rows = I32();
    *cols = I32();
    size_t n = (size_t)*rows * *cols;
    std::vector<double> v(n);
    if (t == "DM") {
      Need(n * 8);
      memcpy(v.data(), d.data() + p, n * 8);
      p += n * 8;
    } else if (t == "FM") {
      Need(n * 4);
      for (size_t i = 0; i < n; i++) { float x; memcpy(&x, d.data() + p, 4); v[i] = x; p += 4; }
    } else {
      VAMD_ERR("unsupported matrix type " << t);
    }
    return v;
  }
  std::vector<double> Vec64() {
    std::string t = Token();
    int n = I32();
    std::vector<double> v(n);
    if (t == "DV") {
      Need((size_t)n * 8);
      memcpy(v.data(), d.data() + p, (size_t)n * 8);
      p += (size_t)n * 8;
    } else if (t == "FV") {
      Need((size_t)n * 4);
      for (int i = 0; i < n; i++) { float x; memcpy(&x, d.data() + p, 4); v[i] = x; p += 4; }
    } else {
      VAMD_ERR("unsupported vector type " << t);
    }
    return v;
  }
  std::vector<double> SpMat64(int* dim) {  // returned full [dim][dim]
    std::string t = Token();
    int n = I32();
    *dim = n;
    std::vector<double> m((size_t)n * n);
    size_t cnt = (size_t)n * (n + 1) / 2, es = t == "DP" ? 8 : 4;
    if (t != "DP" && t != "FP") VAMD_ERR("unsupported packed matrix type " << t);
    Need(cnt * es);
    for (int i = 0; i < n; i++)
      for (int j = 0; j <= i; j++) {
        double x;
        if (es == 8) memcpy(&x, d.data() + p, 8);
        else { float f; memcpy(&f, d.data() + p, 4); x = f; }
        p += es;
        m[(size_t)i * n + j] = m[(size_t)j * n + i] = x;
      }
    return m;
  }
  std::string Line() {
    size_t e = d.find('\n', p);
    if (e == std::string::npos) VAMD_ERR("unterminated line in nnet3 config section");
    std::string s = d.substr(p, e - p);
    p = e + 1;
    return s;
  }
};

enum FieldKind { FK_F, FK_I, FK_B, FK_V, FK_M, FK_IV, FK_FF, FK_II };
const std::map<std::string, FieldKind>& FieldKinds() {
  static const std::map<std::string, FieldKind> k = {
      {"<LearningRateFactor>", FK_F}, {"<MaxChange>", FK_F}, {"<L2Regularize>", FK_F},
      {"<LearningRate>", FK_F}, {"<OrthonormalConstraint>", FK_F}, {"<NumSamplesHistory>", FK_F},
      {"<Alpha>", FK_F}, {"<Epsilon>", FK_F}, {"<TargetRms>", FK_F}, {"<Count>", FK_F},
      {"<DropoutProportion>", FK_F}, {"<BackpropScale>", FK_F}, {"<OderivCount>", FK_F},
      {"<SelfRepairLowerThreshold>", FK_F}, {"<SelfRepairUpperThreshold>", FK_F},
      {"<SelfRepairScale>", FK_F}, {"<ZeroedProportion>", FK_F}, {"<Scale>", FK_F},
      {"<BiasStddev>", FK_F}, {"<ParamStddev>", FK_F},
      // NonlinearComponent self-repair statistics (doubles in newer Kaldi)
      // and ScaleAndOffsetComponent's natural-gradient rank
      {"<NumDimsSelfRepaired>", FK_F}, {"<NumDimsProcessed>", FK_F}, {"<SelfRepairTarget>", FK_F},
      {"<Rank>", FK_I},
      {"<Dim>", FK_I}, {"<BlockDim>", FK_I}, {"<InputDim>", FK_I}, {"<OutputDim>", FK_I},
      {"<RankIn>", FK_I}, {"<RankOut>", FK_I}, {"<UpdatePeriod>", FK_I}, {"<TimePeriod>", FK_I},
      {"<TimeMaskMaxFrames>", FK_I},
      // StatisticsExtractionComponent / StatisticsPoolingComponent (x-vector
      // nnets, nnet3/nnet-general-component.cc [K]; "Varinance" is Kaldi's spelling)
      {"<InputPeriod>", FK_I}, {"<OutputPeriod>", FK_I}, {"<IncludeVarinance>", FK_B},
      {"<LeftContext>", FK_I}, {"<RightContext>", FK_I}, {"<NumLogCountFeatures>", FK_I},
      {"<OutputStddevs>", FK_B}, {"<VarianceFloor>", FK_F},
      {"<IsGradient>", FK_B}, {"<TestMode>", FK_B}, {"<UseNaturalGradient>", FK_B},
      {"<Continuous>", FK_B},
      {"<BiasParams>", FK_V}, {"<StatsMean>", FK_V}, {"<StatsVar>", FK_V}, {"<ValueAvg>", FK_V},
      {"<DerivAvg>", FK_V}, {"<OderivRms>", FK_V}, {"<Scales>", FK_V}, {"<Offsets>", FK_V},
      {"<LinearParams>", FK_M}, {"<Params>", FK_M},
      {"<TimeOffsets>", FK_IV}, {"<AlphaInOut>", FK_FF}, {"<RankInOut>", FK_II}};
  return k;
}

Component ReadComponent(KReader& r) {
  std::string open = r.Token();
  if (open.size() < 3 || open.front() != '<' || open.back() != '>')
    VAMD_ERR("bad component tag " << open);
  Component c;
  c.type = open.substr(1, open.size() - 2);
  std::string close = "</" + c.type + ">";
  const auto& kinds = FieldKinds();
  while (true) {
    std::string tag = r.Token();
    if (tag == close) break;
    auto it = kinds.find(tag);
    if (it == kinds.end()) VAMD_ERR("unknown field " << tag << " in component " << c.type);
    std::string key = tag.substr(1, tag.size() - 2);
    switch (it->second) {
      case FK_F: c.f[key] = r.F32(); break;
      case FK_I: c.i[key] = r.I32(); break;
      case FK_B: c.b[key] = r.Bool(); break;
      case FK_V: c.v[key] = r.Vector(); break;
      case FK_M: c.m[key] = r.Mat(); break;
      case FK_IV: c.time_offsets = r.IntVector(); break;
      case FK_FF: r.F32(); r.F32(); break;
      case FK_II: r.I32(); r.I32(); break;
    }
  }
  return c;
}

// 'component-node name=x component=y input=Append(a, b)' -> key/value map
std::map<std::string, std::string> SplitConfigLine(const std::string& line, std::string* kind) {
  std::string s = Trim(line);
  size_t sp = s.find(' ');
  *kind = s.substr(0, sp);
  std::map<std::string, std::string> kv;
  if (sp == std::string::npos) return kv;
  std::string rest = s.substr(sp + 1);
  size_t i = 0, n = rest.size();
  while (i < n) {
    while (i < n && rest[i] == ' ') ++i;
    if (i >= n) break;
    size_t eq = rest.find('=', i);
    if (eq == std::string::npos) VAMD_ERR("bad nnet3 config line: " << line);
    std::string key = Trim(rest.substr(i, eq - i));
    size_t j = eq + 1;
    int depth = 0;
    while (j < n && (depth > 0 || rest[j] != ' ')) {
      if (rest[j] == '(') ++depth;
      else if (rest[j] == ')') --depth;
      ++j;
    }
    kv[key] = rest.substr(eq + 1, j - eq - 1);
    i = j;
  }
  return kv;
}
}  // namespace

// ---------------------------------------------------------------------------
// descriptor parser
// ---------------------------------------------------------------------------
namespace {
struct DescParser {
  std::vector<std::string> toks;
  size_t k = 0;
  explicit DescParser(const std::string& s) {
    size_t i = 0;
    while (i < s.size()) {
      char c = s[i];
      if (c == ' ' || c == '\t') { ++i; continue; }
      if (c == '(' || c == ')' || c == ',') { toks.push_back(std::string(1, c)); ++i; continue; }
      size_t j = i;
      while (j < s.size() && s[j] != '(' && s[j] != ')' && s[j] != ',' && s[j] != ' ') ++j;
      toks.push_back(s.substr(i, j - i));
      i = j;
    }
  }
  const std::string& Peek() const {
    static const std::string empty;
    return k < toks.size() ? toks[k] : empty;
  }
  std::string Next() {
    if (k >= toks.size()) VAMD_ERR("truncated descriptor");
    return toks[k++];
  }
  void Expect(const std::string& t) {
    std::string g = Next();
    if (g != t) VAMD_ERR("descriptor: expected " << t << " got " << g);
  }
  Desc Parse() {
    std::string name = Next();
    Desc d;
    if (Peek() != "(") {
      d.kind = Desc::NODE;
      d.node = name;
      return d;
    }
    Expect("(");
    if (name == "Append" || name == "Sum") {
      d.kind = name == "Append" ? Desc::APPEND : Desc::SUM;
      d.args.push_back(Parse());
      while (Peek() == ",") { Next(); d.args.push_back(Parse()); }
      Expect(")");
    } else if (name == "Offset") {
      d.kind = Desc::OFFSET;
      d.args.push_back(Parse());
      Expect(",");
      d.t = std::stoi(Next());
      if (Peek() == ",") {
        Next();
        if (std::stoi(Next()) != 0) VAMD_ERR("Offset with nonzero x offset is unsupported");
      }
      Expect(")");
    } else if (name == "Scale") {
      d.kind = Desc::SCALE;
      d.scale = std::stof(Next());
      Expect(",");
      d.args.push_back(Parse());
      Expect(")");
    } else if (name == "ReplaceIndex") {
      d.kind = Desc::REPLACE_INDEX;
      d.args.push_back(Parse());
      Expect(",");
      std::string var = Next();
      if (var != "t") VAMD_ERR("ReplaceIndex only supports t");
      Expect(",");
      d.t = std::stoi(Next());
      Expect(")");
    } else if (name == "Round") {
      d.kind = Desc::ROUND;
      d.args.push_back(Parse());
      Expect(",");
      d.t = std::stoi(Next());
      Expect(")");
    } else if (name == "Const") {
      d.kind = Desc::CONST;
      d.scale = std::stof(Next());
      Expect(",");
      d.dim = std::stoi(Next());
      Expect(")");
    } else if (name == "IfDefined") {
      d.kind = Desc::IFDEFINED;
      d.args.push_back(Parse());
      Expect(")");
    } else {
      VAMD_ERR("unsupported descriptor " << name);
    }
    return d;
  }
};
}  // namespace

Desc ParseDescriptor(const std::string& s) {
  DescParser p(s);
  Desc d = p.Parse();
  if (p.k != p.toks.size()) VAMD_ERR("trailing tokens in descriptor " << s);
  return d;
}

const NnetNode& Nnet::Node(const std::string& n) const {
  auto it = node_index.find(n);
  if (it == node_index.end()) VAMD_ERR("unknown nnet3 node " << n);
  return nodes[it->second];
}

static int ComponentOutputDim(const Component& c) {
  if (c.type == "StatisticsExtractionComponent") {  // [count, sum x (, sum x^2)]
    const int d = c.i.at("InputDim");
    return 1 + d * (c.b.count("IncludeVarinance") && c.b.at("IncludeVarinance") ? 2 : 1);
  }
  if (c.type == "StatisticsPoolingComponent") {  // [log-counts, mean (, stddev)]
    const int n = c.i.count("NumLogCountFeatures") ? c.i.at("NumLogCountFeatures") : 0;
    return c.i.at("InputDim") - 1 + n;
  }
  auto m = c.m.find("LinearParams");
  if (m != c.m.end()) return m->second.rows;
  m = c.m.find("Params");
  if (m != c.m.end()) return m->second.rows;
  auto i = c.i.find("Dim");
  if (i != c.i.end()) return i->second;
  i = c.i.find("OutputDim");
  if (i != c.i.end()) return i->second;
  VAMD_ERR("cannot determine output dim of component type " << c.type);
}

int Nnet::OutputDimOf(const std::string& name) const {
  const NnetNode& nd = Node(name);
  switch (nd.kind) {
    case NnetNode::INPUT: return nd.dim;
    case NnetNode::DIM_RANGE: return nd.dim;
    case NnetNode::OUTPUT: return DescDim(nd.input);
    case NnetNode::COMPONENT: {
      auto it = components.find(nd.component);
      if (it == components.end()) VAMD_ERR("missing component " << nd.component);
      return ComponentOutputDim(it->second);
    }
  }
  return 0;
}

int Nnet::DescDim(const Desc& d) const {
  switch (d.kind) {
    case Desc::NODE: return OutputDimOf(d.node);
    case Desc::APPEND: {
      int s = 0;
      for (auto& a : d.args) s += DescDim(a);
      return s;
    }
    case Desc::CONST: return d.dim;
    default: return DescDim(d.args[0]);
  }
}

void ParseNnet3(KReader& r, size_t size, Nnet* nnet);

void ReadFinalMdl(const std::string& path, TransitionModel* tm, Nnet* nnet) {
  std::ifstream in(path, std::ios::binary);
  if (!in) VAMD_ERR("cannot open " << path);
  std::string data((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  KReader r(data);

  // ---- TransitionModel (hmm/transition-model.cc, hmm/hmm-topology.cc [K])
  r.Expect("<TransitionModel>");
  r.Expect("<Topology>");
  std::vector<int> phones = r.IntVector();
  std::vector<int> phone2idx = r.IntVector();
  int n_entries = r.I32();
  bool is_hmm = true;
  if (n_entries == -1) { is_hmm = false; n_entries = r.I32(); }
  // entries[e][state] -> list of destination states
  std::vector<std::vector<std::vector<int>>> entries(n_entries);
  for (int e = 0; e < n_entries; e++) {
    int ns = r.I32();
    entries[e].resize(ns);
    for (int s = 0; s < ns; s++) {
      r.I32();                // forward pdf class
      if (!is_hmm) r.I32();   // self-loop pdf class
      int nt = r.I32();
      for (int t = 0; t < nt; t++) {
        entries[e][s].push_back(r.I32());
        r.F32();
      }
    }
  }
  r.Expect("</Topology>");
  std::string tt = r.Token();
  bool triples = tt == "<Triples>";
  if (!triples && tt != "<Tuples>") VAMD_ERR("bad transition model tuples tag " << tt);
  int n_tuples = r.I32();
  tm->tid2pdf.assign(1, -1);
  tm->tid2phone.assign(1, 0);
  tm->tid2selfloop.assign(1, 0);
  tm->tid2final.assign(1, 0);
  tm->tid2first.assign(1, 0);
  int max_pdf = -1;
  for (int i = 0; i < n_tuples; i++) {
    int phone = r.I32(), hmm_state = r.I32(), fpdf = r.I32();
    int spdf = triples ? fpdf : r.I32();
    if (phone < 0 || phone >= (int)phone2idx.size() || phone2idx[phone] < 0)
      VAMD_ERR("bad phone " << phone << " in transition model");
    const auto& st = entries[phone2idx[phone]].at(hmm_state);
    for (int dst : st) {
      bool self_loop = dst == hmm_state;
      int pdf = self_loop ? spdf : fpdf;
      tm->tid2pdf.push_back(pdf);
      tm->tid2phone.push_back(phone);
      tm->tid2selfloop.push_back(self_loop ? 1 : 0);
      tm->tid2final.push_back(dst == (int)entries[phone2idx[phone]].size() - 1 ? 1 : 0);
      tm->tid2first.push_back(hmm_state == 0 && !self_loop ? 1 : 0);
      max_pdf = std::max(max_pdf, pdf);
    }
  }
  r.Expect(triples ? "</Triples>" : "</Tuples>");
  r.Expect("<LogProbs>");
  r.Vector();
  r.Expect("</LogProbs>");
  r.Expect("</TransitionModel>");
  tm->num_pdfs = max_pdf + 1;
  ParseNnet3(r, data.size(), nnet);
}

void ReadNnetRaw(const std::string& path, Nnet* nnet) {
  std::ifstream in(path, std::ios::binary);
  if (!in) VAMD_ERR("cannot open " << path);
  std::string data((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  KReader r(data);
  ParseNnet3(r, data.size(), nnet);
}

std::vector<float> ReadKaldiVectorFloat(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) VAMD_ERR("cannot open " << path);
  std::string d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  KReader r(d);
  return r.Vector();
}

Matrix ReadKaldiMatrixFloat(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) VAMD_ERR("cannot open " << path);
  std::string d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  KReader r(d);
  return r.Mat();
}

// nnet3 (nnet3/nnet-nnet.cc, nnet3/am-nnet-simple.cc [K]): config lines,
// components, then AmNnetSimple's context / priors when present
void ParseNnet3(KReader& r, size_t size, Nnet* nnet) {
  r.Expect("<Nnet3>");
  r.Line();  // remainder of the token's line
  nnet->nodes.clear();
  nnet->node_index.clear();
  while (true) {
    std::string ln = r.Line();
    if (Trim(ln).empty()) break;
    std::string kind;
    auto kv = SplitConfigLine(ln, &kind);
    NnetNode nd;
    nd.name = kv["name"];
    if (kind == "input-node") {
      nd.kind = NnetNode::INPUT;
      nd.dim = std::stoi(kv["dim"]);
    } else if (kind == "component-node") {
      nd.kind = NnetNode::COMPONENT;
      nd.component = kv["component"];
      nd.input = ParseDescriptor(kv["input"]);
    } else if (kind == "output-node") {
      nd.kind = NnetNode::OUTPUT;
      nd.input = ParseDescriptor(kv["input"]);
    } else if (kind == "dim-range-node") {
      nd.kind = NnetNode::DIM_RANGE;
      nd.src = kv["input-node"];
      nd.dim_offset = std::stoi(kv["dim-offset"]);
      nd.dim = std::stoi(kv["dim"]);
    } else {
      VAMD_ERR("unsupported nnet3 config line kind " << kind);
    }
    nnet->node_index[nd.name] = (int)nnet->nodes.size();
    nnet->nodes.push_back(std::move(nd));
  }
  r.Expect("<NumComponents>");
  int nc = r.I32();
  for (int c = 0; c < nc; c++) {
    r.Expect("<ComponentName>");
    std::string name = r.Token();
    nnet->components[name] = ReadComponent(r);
  }
  r.Expect("</Nnet3>");
  if (r.p < size && r.PeekToken() == "<LeftContext>") {
    r.Expect("<LeftContext>");
    nnet->left_context = r.I32();
    r.Expect("<RightContext>");
    nnet->right_context = r.I32();
    if (r.p < size && r.PeekToken() == "<Priors>") {
      r.Expect("<Priors>");
      std::vector<float> pri = r.Vector();
      if (!pri.empty()) VAMD_WARN("non-empty priors ignored (chain models have none)");
    }
  }
}

// ---------------------------------------------------------------------------
// OpenFST reader
// ---------------------------------------------------------------------------
namespace {
constexpr int32_t kFstMagic = 2125659606;
constexpr int32_t kSymMagic = 2125658996;

struct BReader {
  std::string d;
  size_t p = 0;
  void Need(size_t n) const {
    if (p + n > d.size()) VAMD_ERR("unexpected end of FST file");
  }
  template <class T> T Get() {
    Need(sizeof(T));
    T v;
    memcpy(&v, d.data() + p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string Str() {
    int32_t n = Get<int32_t>();
    Need(n);
    std::string s = d.substr(p, n);
    p += n;
    return s;
  }
};

void ReadSymtab(BReader& r, std::map<int, std::string>* out) {
  if (r.Get<int32_t>() != kSymMagic) VAMD_ERR("bad symbol table magic in FST");
  r.Str();
  r.Get<int64_t>();
  int64_t n = r.Get<int64_t>();
  for (int64_t i = 0; i < n; i++) {
    std::string sym = r.Str();
    int64_t key = r.Get<int64_t>();
    if (out) (*out)[(int)key] = sym;
  }
}
}  // namespace

namespace {
constexpr int32_t kAddOnMagic = 446681434;

// LOUDS n-gram FST body (OpenFST extensions/ngram NGramFstImpl::Init layout):
// uint64 num_states, num_futures, num_final; context bitmap (2n+1 bits),
// future bitmap (num_futures+n+1 bits), final bitmap (n bits), each in 64-bit
// words with bit i at word i/64, position i%64; int32 context words [n+1],
// future words [num_futures]; padding to 4 bytes; float backoff [n+1], final
// costs [num_final], future costs [num_futures+1].
void ParseNgramBody(BReader& r, HostFst* f, const std::string& path) {
  const uint64_t n = r.Get<uint64_t>(), nfut = r.Get<uint64_t>(), nfin = r.Get<uint64_t>();
  if (n < 2 || n > (1ull << 31) || nfut > (1ull << 34) || nfin > n) VAMD_ERR("malformed ngram FST " << path);
  auto words64 = [](uint64_t bits) { return (bits + 63) / 64; };
  const uint64_t cbits = 2 * n + 1, fbits = nfut + n + 1;
  std::vector<uint64_t> ctx(words64(cbits)), fut(words64(fbits)), fin(words64(n));
  for (auto& v : ctx) v = r.Get<uint64_t>();
  for (auto& v : fut) v = r.Get<uint64_t>();
  for (auto& v : fin) v = r.Get<uint64_t>();
  std::vector<int32_t> cwords(n + 1), fwords(nfut);
  for (auto& v : cwords) v = r.Get<int32_t>();
  for (auto& v : fwords) v = r.Get<int32_t>();
  std::vector<float> backoff(n + 1), finals(nfin), fprob(nfut + 1);
  for (auto& v : backoff) v = r.Get<float>();
  for (auto& v : finals) v = r.Get<float>();
  for (auto& v : fprob) v = r.Get<float>();
  auto bit = [](const std::vector<uint64_t>& b, uint64_t i) { return (b[i >> 6] >> (i & 63)) & 1; };
  // context tree (LOUDS with super-root "10"): node ids in level order; the
  // degree sequence of node k (1^d 0) follows the super-root's
  if (!(bit(ctx, 0) == 1 && bit(ctx, 1) == 0)) VAMD_ERR("malformed ngram FST context " << path);
  std::vector<int> parent(n, -1), first_child(n, 0), num_children(n, 0);
  {
    uint64_t pos = 2, next = 1;
    for (uint64_t k = 0; k < n; k++) {
      first_child[k] = (int)next;
      while (pos < cbits && bit(ctx, pos)) {
        if (next >= n) VAMD_ERR("malformed ngram FST context " << path);
        parent[next++] = (int)k;
        num_children[k]++;
        pos++;
      }
      if (pos >= cbits) VAMD_ERR("malformed ngram FST context " << path);
      pos++;  // the 0 that ends node k's degree sequence
    }
    if (next != n || num_children[0] == 0)
      VAMD_ERR("malformed ngram FST context " << path);
  }
  // futures: a leading 0, then 1^k 0 per state
  std::vector<int64_t> fut_begin(n + 1, 0);
  {
    if (bit(fut, 0) != 0) VAMD_ERR("malformed ngram FST futures " << path);
    uint64_t pos = 1, ones = 0;
    for (uint64_t s = 0; s < n; s++) {
      fut_begin[s] = (int64_t)ones;
      while (pos < fbits && bit(fut, pos)) { ones++; pos++; }
      if (pos >= fbits) VAMD_ERR("malformed ngram FST futures " << path);
      pos++;
    }
    fut_begin[n] = (int64_t)ones;
    if (ones != nfut) VAMD_ERR("malformed ngram FST futures " << path);
  }
  // child of node k labelled w (children are sorted by label), or -1
  auto child = [&](int k, int w) {
    const int32_t* b = cwords.data() + first_child[k];
    const int32_t* e = b + num_children[k];
    const int32_t* it = std::lower_bound(b, e, w);
    return (it == e || *it != w) ? -1 : first_child[k] + (int)(it - b);
  };
  std::vector<int> ctx_words;  // labels from the state's node up to the root
  f->start = 1;
  f->final_cost.assign(n, std::numeric_limits<float>::infinity());
  f->row.assign(n + 1, 0);
  f->ilabel.clear(); f->olabel.clear(); f->weight.clear(); f->nextstate.clear();
  uint64_t nf = 0;
  for (uint64_t s = 0; s < n; s++) {
    f->row[s] = (int64_t)f->ilabel.size();
    if (bit(fin, s)) f->final_cost[s] = finals[nf++];
    if (s != 0) {  // backoff: the parent context (oldest word dropped)
      f->ilabel.push_back(0); f->olabel.push_back(0);
      f->weight.push_back(backoff[s]); f->nextstate.push_back(parent[s]);
    }
    ctx_words.clear();
    for (int k = (int)s; k != 0; k = parent[k]) ctx_words.push_back(cwords[k]);
    for (int64_t i = fut_begin[s]; i < fut_begin[s + 1]; i++) {
      const int w = fwords[i];
      // NGramFstImpl::Transition: the root's child w, then down the
      // state's context from its most recent word while children exist
      int node = child(0, w);
      if (node < 0) {
        node = 0;
      } else {
        for (int j = (int)ctx_words.size() - 1; j >= 0 && num_children[node] > 0; j--) {
          const int c = child(node, ctx_words[j]);
          if (c < 0) break;
          node = c;
        }
      }
      f->ilabel.push_back(w); f->olabel.push_back(w);
      f->weight.push_back(fprob[i]); f->nextstate.push_back(node);
    }
  }
  f->row[n] = (int64_t)f->ilabel.size();
  if (nf != nfin) VAMD_ERR("malformed ngram FST finals " << path);
}

void ParseFst(BReader& r, HostFst* f, const std::string& path, int depth) {
  if (r.Get<int32_t>() != kFstMagic) VAMD_ERR(path << " is not an OpenFST binary file");
  std::string ftype = r.Str(), atype = r.Str();
  if (atype != "standard") VAMD_ERR("unsupported arc type " << atype << " in " << path);
  r.Get<int32_t>();  // version
  int32_t flags = r.Get<int32_t>();
  r.Get<uint64_t>();  // properties
  int64_t start = r.Get<int64_t>(), ns = r.Get<int64_t>(), na = r.Get<int64_t>();
  if (flags & 1) ReadSymtab(r, nullptr);
  if (flags & 2) ReadSymtab(r, &f->osyms);
  f->ilabel.clear(); f->olabel.clear(); f->weight.clear(); f->nextstate.clear();
  f->final_cost.clear(); f->row.clear();
  if (ftype == "const") {
    if (ns < 0 || na < 0) VAMD_ERR("bad const FST header in " << path);
    if (flags & 4) r.p = (r.p + 15) / 16 * 16;
    f->final_cost.resize(ns);
    f->row.resize(ns + 1);
    for (int64_t s = 0; s < ns; s++) {
      f->final_cost[s] = r.Get<float>();
      f->row[s] = r.Get<uint32_t>();
      r.Get<uint32_t>();
      r.Get<uint32_t>();
      r.Get<uint32_t>();
    }
    f->row[ns] = na;
    if (flags & 4) r.p = (r.p + 15) / 16 * 16;
    f->ilabel.resize(na); f->olabel.resize(na); f->weight.resize(na); f->nextstate.resize(na);
    for (int64_t a = 0; a < na; a++) {
      f->ilabel[a] = r.Get<int32_t>();
      f->olabel[a] = r.Get<int32_t>();
      f->weight[a] = r.Get<float>();
      f->nextstate[a] = r.Get<int32_t>();
    }
    f->start = (int)start;
  } else if (ftype == "vector") {
    f->row.push_back(0);
    for (int64_t s = 0; ns < 0 ? r.p < r.d.size() : s < ns; s++) {
      f->final_cost.push_back(r.Get<float>());
      int64_t n = r.Get<int64_t>();
      for (int64_t a = 0; a < n; a++) {
        f->ilabel.push_back(r.Get<int32_t>());
        f->olabel.push_back(r.Get<int32_t>());
        f->weight.push_back(r.Get<float>());
        f->nextstate.push_back(r.Get<int32_t>());
      }
      f->row.push_back((int64_t)f->ilabel.size());
    }
    f->start = (int)start;
  } else if (ftype == "ngram") {
    ParseNgramBody(r, f, path);
  } else if (ftype == "olabel_lookahead" && depth == 0) {
    if (r.Get<int32_t>() != kAddOnMagic) VAMD_ERR("bad add-on header in " << path);
    std::map<int, std::string> outer = std::move(f->osyms);
    ParseFst(r, f, path, depth + 1);  // the contained FST; the add-on data is not needed
    if (f->osyms.empty()) f->osyms = std::move(outer);
  } else {
    VAMD_ERR("unsupported FST type '" << ftype << "' in " << path);
  }
  const int64_t S = f->NumStates();
  if (S > 0 && (f->start < 0 || f->start >= S)) VAMD_ERR("bad start state in " << path);
  for (int64_t a = 0; a < f->NumArcs(); a++)
    if (f->nextstate[a] < 0 || f->nextstate[a] >= S) VAMD_ERR("arc to invalid state in " << path);
}
}  // namespace

void ReadFst(const std::string& path, HostFst* f) {
  BReader r;
  {
    std::ifstream in(path, std::ios::binary);
    if (!in) VAMD_ERR("cannot open " << path);
    r.d.assign((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  }
  *f = HostFst();
  ParseFst(r, f, path, 0);
}

void ToGraph(const HostFst& f, Graph* g, const std::string& what) {
  const int64_t S = f.NumStates(), A = f.NumArcs();
  if (S == 0) VAMD_ERR(what << " has no states");
  g->start = f.start;
  g->final_cost = f.final_cost;
  g->osyms = f.osyms;
  g->arc_begin.assign(S + 1, 0);
  g->eps_begin.assign(S, 0);
  g->ilabel.resize(A); g->olabel.resize(A); g->weight.resize(A); g->nextstate.resize(A);
  int64_t o = 0;
  for (int64_t s = 0; s < S; s++) {  // emitting arcs first (stable), then epsilon-input arcs
    g->arc_begin[s] = o;
    for (int pass = 0; pass < 2; pass++) {
      if (pass == 1) g->eps_begin[s] = o;
      for (int64_t a = f.row[s]; a < f.row[s + 1]; a++) {
        if ((f.ilabel[a] == 0) != (pass == 1)) continue;
        g->ilabel[o] = f.ilabel[a]; g->olabel[o] = f.olabel[a];
        g->weight[o] = f.weight[a]; g->nextstate[o] = f.nextstate[a];
        ++o;
      }
    }
  }
  g->arc_begin[S] = o;
  g->lazy_row = f.lazy_row;
  g->lazy_next = f.lazy_next;
  g->lazy_ids = f.lazy_ids;
}

void ReadFstGraph(const std::string& path, Graph* g) {
  HostFst f;
  ReadFst(path, &f);
  ToGraph(f, g, path);
}

void ReadSymbolTable(const std::string& path, SymbolTable* t) {
  std::ifstream in(path);
  if (!in) VAMD_ERR("cannot open symbol table " << path);
  std::string sym;
  long id;
  std::string ln;
  while (std::getline(in, ln)) {
    std::istringstream ss(ln);
    if (!(ss >> sym >> id)) continue;
    t->id2sym[(int)id] = sym;
    t->sym2id[sym] = (int)id;
  }
}

// ---------------------------------------------------------------------------
// i-vector extractor directory (src/model.cc:247-263 file set)
// ---------------------------------------------------------------------------
std::vector<double> ReadKaldiMatrixFile(const std::string& path, int* rows, int* cols) {
  std::ifstream f(path, std::ios::binary);
  if (!f) VAMD_ERR("cannot open " << path);
  std::string d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  KReader r(d);
  return r.Mat64(rows, cols);
}

void ReadIvectorModel(const std::string& dir, IvectorModel* m) {
  auto slurp = [](const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) VAMD_ERR("cannot open " << path);
    return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  };
  for (auto& [k, v] : ReadConfigFile(dir + "/splice.conf")) {
    if (k == "left-context") m->left = std::stoi(v);
    else if (k == "right-context") m->right = std::stoi(v);
  }
  if (FileExists(dir + "/online_cmvn.conf"))
    for (auto& [k, v] : ReadConfigFile(dir + "/online_cmvn.conf")) {
      if (k == "cmn-window") m->cmn_window = std::stoi(v);
      else if (k == "global-frames") m->global_frames = std::stoi(v);
      else if (k == "norm-vars" || k == "normalize-variance") {
        if (v == "true") VAMD_ERR("online CMVN with variance normalization is not supported");
      } else {
        VAMD_WARN("ignoring online CMVN option --" << k);
      }
    }
  {
    std::string d = slurp(dir + "/final.mat");
    KReader r(d);
    m->lda = r.Mat();
  }
  {
    std::string d = slurp(dir + "/global_cmvn.stats");
    KReader r(d);
    int rows, cols;
    m->cmvn = r.Mat64(&rows, &cols);
    if (rows != 2) VAMD_ERR("bad global_cmvn.stats");
    m->feat_dim = cols - 1;
  }
  {
    std::string d = slurp(dir + "/final.dubm");
    KReader r(d);
    r.Expect("<DiagGMM>");
    r.Expect("<GCONSTS>");
    m->gconsts = r.Vector();
    r.Expect("<WEIGHTS>");
    r.Vector();
    r.Expect("<MEANS_INVVARS>");
    Matrix mi = r.Mat();
    r.Expect("<INV_VARS>");
    Matrix iv = r.Mat();
    m->num_gauss = mi.rows;
    m->lda_dim = mi.cols;
    m->means_invvars = mi.data;
    m->inv_vars = iv.data;
  }
  {
    std::string d = slurp(dir + "/final.ie");
    KReader r(d);
    r.Expect("<IvectorExtractor>");
    r.Expect("<w>");
    int a, b;
    r.Mat64(&a, &b);
    r.Expect("<w_vec>");
    r.Vec64();
    r.Expect("<M>");
    const int G = r.I32();
    if (G != m->num_gauss) VAMD_ERR("final.ie / final.dubm Gaussian count mismatch");
    for (int g = 0; g < G; g++) {
      int rows, cols;
      std::vector<double> M = r.Mat64(&rows, &cols);
      if (rows != m->lda_dim) VAMD_ERR("final.ie feature dim mismatch");
      m->ivec_dim = cols;
      m->M.insert(m->M.end(), M.begin(), M.end());
    }
    r.Expect("<SigmaInv>");
    for (int g = 0; g < G; g++) {
      int n;
      std::vector<double> S = r.SpMat64(&n);
      m->sigma_inv.insert(m->sigma_inv.end(), S.begin(), S.end());
    }
    r.Expect("<IvectorOffset>");
    m->prior_offset = r.F64();
  }
  const int D = m->lda_dim, S = m->ivec_dim, G = m->num_gauss, QS = S * (S + 1) / 2;
  if (m->lda.rows != D) VAMD_ERR("final.mat output dim != UBM dim");
  const int K = (m->left + m->right + 1) * m->feat_dim;
  if (m->lda.cols != K && m->lda.cols != K + 1) VAMD_ERR("final.mat input dim mismatch");
  // derived terms, IvectorExtractor::ComputeDerivedVars (order shared with oracle.c)
  m->sigma_inv_m.assign((size_t)G * D * S, 0.0);
  m->U.assign((size_t)G * QS, 0.0);
  for (int g = 0; g < G; g++) {
    const double* M = m->M.data() + (size_t)g * D * S;
    const double* SI = m->sigma_inv.data() + (size_t)g * D * D;
    double* sm = m->sigma_inv_m.data() + (size_t)g * D * S;
    for (int d = 0; d < D; d++)
      for (int s2 = 0; s2 < S; s2++) {
        double a = 0.0;
        for (int e = 0; e < D; e++) a = a + SI[(size_t)d * D + e] * M[(size_t)e * S + s2];
        sm[(size_t)d * S + s2] = a;
      }
    double* u = m->U.data() + (size_t)g * QS;
    for (int i = 0; i < S; i++)
      for (int j = 0; j <= i; j++) {
        double a = 0.0;
        for (int d = 0; d < D; d++) a = a + M[(size_t)d * S + i] * sm[(size_t)d * S + j];
        u[(size_t)i * (i + 1) / 2 + j] = a;
      }
  }
  m->log_min_post = (float)std::log((double)m->min_post);
  VAMD_LOG("i-vector extractor: dim " << S << ", " << G << " Gaussians, LDA " << m->lda.rows << "x"
                                      << m->lda.cols << ", prior offset " << m->prior_offset);
}

}  // namespace vamd
