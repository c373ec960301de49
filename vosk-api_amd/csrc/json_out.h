// Minimal JSON value whose dump() reproduces the byte format of the
// reference's SimpleJSON writer (src/json.h:343-380): objects with keys in
// sorted (std::map) order, "{\n" + pad + "\"key\" : " + value, two-space
// indentation per depth, arrays as "[a, b]", floats via std::to_string (six
// decimals), strings escaped as json_escape (src/json.h:34-48).
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace vamd {

class Json {
 public:
  enum Kind { NUL, OBJECT, ARRAY, STRING, FLOAT, INT, BOOL };
  Json() = default;
  static Json Str(const std::string& s) { Json j; j.kind_ = STRING; j.s_ = s; return j; }
  static Json Float(double d) { Json j; j.kind_ = FLOAT; j.d_ = d; return j; }
  static Json Int(long i) { Json j; j.kind_ = INT; j.i_ = i; return j; }
  Json& operator[](const std::string& k) {
    if (kind_ != OBJECT) { kind_ = OBJECT; map_.clear(); }
    return map_[k];
  }
  void Append(const Json& v) {
    if (kind_ != ARRAY) { kind_ = ARRAY; list_.clear(); }
    list_.push_back(v);
  }

  std::string Dump(int depth = 1, const std::string& tab = "  ") const {
    std::string pad;
    for (int i = 0; i < depth; ++i) pad += tab;
    switch (kind_) {
      case NUL: return "null";
      case OBJECT: {
        std::string s = "{\n";
        bool skip = true;
        for (auto& p : map_) {
          if (!skip) s += ",\n";
          s += pad + "\"" + p.first + "\" : " + p.second.Dump(depth + 1, tab);
          skip = false;
        }
        s += "\n" + pad.erase(0, 2) + "}";
        return s;
      }
      case ARRAY: {
        std::string s = "[";
        bool skip = true;
        for (auto& p : list_) {
          if (!skip) s += ", ";
          s += p.Dump(depth + 1, tab);
          skip = false;
        }
        return s + "]";
      }
      case STRING: return "\"" + Escape(s_) + "\"";
      case FLOAT: return std::to_string(d_);
      case INT: return std::to_string(i_);
      case BOOL: return b_ ? "true" : "false";
    }
    return "";
  }

  static std::string Escape(const std::string& str) {
    std::string out;
    for (char c : str) {
      switch (c) {
        case '\"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\b': out += "\\b"; break;
        case '\f': out += "\\f"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        default: out += c;
      }
    }
    return out;
  }

 private:
  Kind kind_ = NUL;
  std::string s_;
  double d_ = 0;
  long i_ = 0;
  bool b_ = false;
  std::map<std::string, Json> map_;
  std::vector<Json> list_;
};

}  // namespace vamd
