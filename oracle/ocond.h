// ORACLE — test infrastructure only (see ojson.h header).
//
// Conditions of validate.deny and rule preconditions, restated from
//   pkg/engine/variables/evaluate.go:11-83          (Evaluate / EvaluateConditions / any-all / old list)
//   pkg/engine/variables/operator/*.go              (Equal, NotEqual, In, AnyIn, AllIn, NotIn, AnyNotIn, AllNotIn,
//                                                    numeric >, >=, <, <= incl. duration / quantity / semver)
//   pkg/utils/api/json.go:30-85                     (ApiextensionsJsonToKyvernoConditions)
//   pkg/engine/variables/vars.go:352-431            (substituteVariablesIfAny, restricted: see below)
//   pkg/engine/validation.go:276-290,437-479        (preconditions -> skip, validateDeny, getDenyMessage)
//
// Variable support is the subset the device compiles: a string that is exactly one `{{ <expr> }}` where <expr> is
// a dotted chain of JMESPath identifiers from request.object, or an expression of the JMESPath subset of ojmes.h
// (projections, multi-select lists, `||` literals, keys()) from request.object / request.operation / element.
// Anything else containing `{{` or `$(` is reported unsupported (those rules stay on the reference's CPU engine).
#pragma once
#include <string>

#include "ojson.h"

namespace orc {

// Operator handler result for one condition (operator.CreateOperatorHandler(op).Evaluate(key, value)).
// Throws RefPanic where the reference panics (NotIn/In with a non-string element in a key list).
bool evaluate_condition(const oj::VP& key, const std::string& op, const oj::VP& value);

// The `key`/`value` as Condition.GetKey()/GetValue() hands them to the operator: the condition document is
// json.Marshal'ed and decoded again through apimachinery util/json (integral numbers -> int64).
oj::VP condition_operand(const oj::VP& v);

enum class CondOutcome { True, False, Error, Unsupported };

struct CondResult {
  CondOutcome r = CondOutcome::False;
  std::string err;            // Error: variable resolution error text (without the caller's prefix)
  bool err_unpinned = false;  // several variables failed: which one the reference reports depends on Go map order
};

// SubstituteAll(ctx, conditions) + TransformConditions + EvaluateConditions for a background-scan JSON context
// whose request.object is `resource`. `conditions` is the raw JSON of rule.preconditions / deny.conditions
// (nullptr when absent).
CondResult eval_conditions(const oj::VP& conditions, const oj::VP& resource);
// same inside a foreach: `element` / `elementIndex` bound (validation.go:383-413 addElementToContext)
CondResult eval_conditions_element(const oj::VP& conditions, const oj::VP& resource, const oj::VP& element,
                                   int64_t index);
bool conditions_supported_element(const oj::VP& conditions);

// getDenyMessage's SubstituteAll(msg) (validation.go:466-479) for messages whose variables are request.object
// references; *unpinned when the message uses anything else (other variables, references, escapes).
std::string render_message(const std::string& msg, const oj::VP& resource, bool* unpinned);
int substitute_message(const std::string& msg, const oj::VP& resource, std::string* out);

// true when every string in `conditions` is either variable-free or exactly one supported request.object
// reference (the device subset); false -> the rule is CPU fallback
bool conditions_supported(const oj::VP& conditions);

// blang/semver v4 Parse + Compare (numeric operators on strings that are none of duration/quantity/number)
bool semver_parse_cmp(const std::string& a, const std::string& b, int* cmp, bool* b_ok);
bool semver_ok(const std::string& s);

}  // namespace orc
