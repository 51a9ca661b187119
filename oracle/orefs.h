// ORACLE — test infrastructure only (see ojson.h header).
#pragma once
#include <string>

#include "ojson.h"

namespace orc {

// variables.substituteReferences over one pattern / anyPattern document (pkg/engine/variables/vars.go:244-346).
// ok = false: the reference returns an error (`err` is its text, as validation.go:295-296 wraps it); nd = true:
// the result depends on Go map iteration order (several elements on the referenced path, or a renamed key that
// collides with another key).
struct RefResult {
  bool ok = true;
  bool nd = false;
  bool err_unpinned = false;  // the error text embeds a Go %v rendering the restatement does not reproduce
  std::string err;
  oj::VP doc;
};
RefResult substitute_references(const oj::VP& doc);
bool has_references(const oj::VP& v);
std::string form_absolute_path(const std::string& ref, const std::string& at);  // any `$(` in a key or string leaf

}  // namespace orc
