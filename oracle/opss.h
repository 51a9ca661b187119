// ORACLE — test infrastructure only (see ojson.h header).
#pragma once
#include <string>
#include <vector>

#include "ojson.h"

namespace orc {

struct CheckResult {
  bool allowed;
  std::string reason, detail;
};
struct PSSResult {
  std::string id;
  CheckResult r;
};
struct PSSEval {
  bool ok = false;            // evaluated
  std::string error;          // version parse error (rule error)
  std::string decode_error;   // typed decode failure (rule error)
  bool allowed = false;
  bool order_nondeterministic = false;  // excludes => Go-map ordered results
  std::vector<PSSResult> checks;
};

PSSEval pss_evaluate(const oj::VP& podSecurity, const oj::VP& meta, const oj::VP& spec, const oj::VP& outerMeta = nullptr);
std::string format_checks_print(const std::vector<PSSResult>& checks);
bool pss_version_ok(const std::string& v);

}  // namespace orc
