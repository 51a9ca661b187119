// ORACLE — test infrastructure only (see ojson.h header).
#pragma once
#include <string>

#include "ojson.h"

namespace orc {

// Error value of the reference's walk. typed = anchor.validateAnchorError with code;
// untyped errors are classified by substring (pkg/engine/anchor/error.go:64-75).
struct Err {
  bool present = false;
  int code = -1;  // -1 untyped, 0 conditional, 1 global, 2 negation
  std::string msg;
  static Err none() { return Err(); }
  static Err make(const std::string& m, int c = -1) { Err e; e.present = true; e.code = c; e.msg = m; return e; }
};

bool is_conditional_err(const Err& e);
bool is_global_err(const Err& e);
bool is_negation_err(const Err& e);

// Thrown for conditions where the reference panics (type assertions in wildcards.go:118,126 ...).
struct RefPanic { std::string what; };

// Evaluation context flags (nondeterminism of the reference; Go map iteration order).
struct EvalFlags {
  bool nondeterministic = false;
};

// pkg/engine/validate/validate.go:31-56 MatchPattern -> PatternError{Err, Path, Skip} or none
struct PatternResult {
  bool ok = true;     // nil error
  bool skip = false;
  std::string path;
  std::string err;    // PatternError.Error()
};

PatternResult match_pattern(const oj::VP& resource, const oj::VP& pattern, EvalFlags& fl);

// pkg/engine/pattern/pattern.go:26 Validate(value, pattern)
bool pattern_validate(const oj::VP& value, const oj::VP& pattern);

}  // namespace orc

namespace orc {
struct RawWalk {
  std::string path;
  bool err = false;
  std::string msg;
};
bool leaf_fn(const std::string& fn, const oj::VP& v, const oj::VP& p, const std::string& op);
RawWalk validate_entry(const std::string& entry, const oj::VP& res, const oj::VP& pat, EvalFlags& fl);
}  // namespace orc

namespace orc {
bool is_in_range_pattern(const std::string& p);
}  // namespace orc

namespace orc {
std::string remove_anchors_from_path(const std::string& str);
std::string anchor_probe(const std::string& op, const std::string& a, const std::string& b);
}  // namespace orc
