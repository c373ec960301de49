// Common helpers for the MI355X-native Vosk hot path (libvosk.so).
#pragma once

#include <cstdint>
#include <cstdio>
#include <sstream>
#include <stdexcept>
#include <string>

namespace vamd {

// Log levels follow vosk_set_log_level (src/vosk_api.cc:176-179 -> Kaldi
// verbosity): <0 silences info, 0 = info (default), >0 = verbose.
int LogLevel();
void SetLogLevel(int level);
void LogMessage(const char* kind, const std::string& msg);

struct Fatal : std::runtime_error {
  explicit Fatal(const std::string& m) : std::runtime_error(m) {}
};

}  // namespace vamd

#define VAMD_LOG(msg)                                              \
  do {                                                             \
    if (::vamd::LogLevel() >= 0) {                                 \
      std::ostringstream _os; _os << msg;                          \
      ::vamd::LogMessage("LOG", _os.str());                        \
    }                                                              \
  } while (0)
#define VAMD_LOG_VERBOSE(msg)                                      \
  do {                                                             \
    if (::vamd::LogLevel() > 0) {                                  \
      std::ostringstream _os; _os << msg;                          \
      ::vamd::LogMessage("VLOG[1]", _os.str());                    \
    }                                                              \
  } while (0)
#define VAMD_WARN(msg)                                             \
  do {                                                             \
    if (::vamd::LogLevel() >= -1) {                                \
      std::ostringstream _os; _os << msg;                          \
      ::vamd::LogMessage("WARNING", _os.str());                    \
    }                                                              \
  } while (0)
#define VAMD_ERR(msg)                                              \
  do {                                                             \
    std::ostringstream _os; _os << msg;                            \
    ::vamd::LogMessage("ERROR", _os.str());                        \
    throw ::vamd::Fatal(_os.str());                                \
  } while (0)
#define VAMD_CHECK(cond, msg)                                      \
  do { if (!(cond)) VAMD_ERR("check failed: " #cond ": " << msg); } while (0)
