// ORACLE — test infrastructure only (see ojson.h header).
//
// JMESPath for the variables of conditions and foreach lists: a restatement of github.com/jmespath/go-jmespath
// (parser.go Pratt parser with its binding powers, interpreter.go node semantics) for the node kinds the chart and
// best-practices policies use -- fields, sub-expressions, multi-select lists, flatten projections, `||`, raw
// string / JSON literals, `@` and the keys() function -- plus the kyverno/go-jmespath fork's missing-key error.
// Neither module is vendored under the reference (go.mod:27,342). The fork behaviour is pinned by the reference's
// own fixtures: a plain field chain whose key is missing from a map fails with NotFoundError "Unknown key "k" in
// path" (pkg/engine/validation_test.go:1939); inside projections, multi-select lists and `||` a missing key is null
// (test/cli/apply + cmd/cli/kubectl-kyverno/apply/apply_command_test.go: `element.securityContext.capabilities.drop
// || ''` and `request.object.spec.[ephemeralContainers, initContainers, containers][]` on Pods without those keys
// give Warn 2 / Error 0). Anything outside the restated subset throws JmesUnsupported.
#pragma once
#include <string>

#include "ojson.h"

namespace orc {

struct JmesUnsupported { std::string why; };
struct JmesNotFound { std::string key; };
struct JmesError { std::string msg; };  // run-time error (e.g. keys() of a non-object)

// true when `expr` parses within the restated subset and starts at one of the roots the background-scan JSON
// context holds for a rule: request.object, request.operation, element (foreach)
bool jmes_supported(const std::string& expr, bool allow_element);

// ctx.Query(expr) over the background-scan JSON context {"request": {"object": resource, "operation": "CREATE"},
// "element": element, "elementIndex": index} (numbers float64, as encoding/json decodes the context). element may be
// nullptr outside foreach. Throws JmesNotFound / JmesError / JmesUnsupported.
oj::VP jmes_query(const std::string& expr, const oj::VP& resource, const oj::VP& element, int64_t index);

// the JSON context's view of a value (encoding/json: every number float64), e.g. a foreach element
oj::VP json_floats(const oj::VP& v);

}  // namespace orc
