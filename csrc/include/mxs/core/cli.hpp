// Minimal command-line parser for the apps: positional arguments (the
// reference's argv[1]/argv[2] contract is kept verbatim) plus --key value,
// --key=value and boolean --flag options.
#pragma once

#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace mxs {

class Cli {
 public:
  // `flags`: option names that take no value.
  Cli(int argc, char** argv, std::set<std::string> flags = {}) : flags_(std::move(flags)) {
    prog_ = argc > 0 ? argv[0] : "";
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.rfind("--", 0) == 0) {
        std::string k = a.substr(2), v;
        const auto eq = k.find('=');
        if (eq != std::string::npos) {
          v = k.substr(eq + 1);
          k = k.substr(0, eq);
        } else if (!flags_.count(k) && i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) {
          v = argv[++i];
        } else {
          v = "1";
        }
        opts_[k] = v;
      } else {
        pos_.push_back(a);
      }
    }
  }
  bool has(const std::string& k) const { return opts_.count(k) != 0; }
  std::string get(const std::string& k, const std::string& def = "") const {
    auto it = opts_.find(k);
    return it == opts_.end() ? def : it->second;
  }
  long long get_int(const std::string& k, long long def) const {
    auto it = opts_.find(k);
    return it == opts_.end() ? def : std::atoll(it->second.c_str());
  }
  double get_double(const std::string& k, double def) const {
    auto it = opts_.find(k);
    return it == opts_.end() ? def : std::atof(it->second.c_str());
  }
  bool flag(const std::string& k) const {
    auto it = opts_.find(k);
    return it != opts_.end() && it->second != "0" && it->second != "false";
  }
  const std::vector<std::string>& positional() const { return pos_; }
  const std::string& program() const { return prog_; }

 private:
  std::set<std::string> flags_;
  std::map<std::string, std::string> opts_;
  std::vector<std::string> pos_;
  std::string prog_;
};

// "WxH" -> {W, H}; {0, 0} when malformed.
inline std::pair<long long, long long> parse_wxh(const std::string& s) {
  const auto p = s.find_first_of("xX");
  if (p == std::string::npos) return {0, 0};
  return {std::atoll(s.substr(0, p).c_str()), std::atoll(s.substr(p + 1).c_str())};
}

}  // namespace mxs
