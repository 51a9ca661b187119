// ORACLE — test infrastructure only (see ojson.h header). Whole-object typed decode of getSpec (see otyped.cpp).
#pragma once
#include <string>

#include "ojson.h"

namespace orc {

struct TypedDecodeError { std::string msg; };

// "" when json.Unmarshal of `resource` into the getSpec target of `kind` (corev1.Pod, appsv1.Deployment for the
// workload kinds, batchv1.CronJob) succeeds (or the kind has none), else the (parity-unpinned) error text
// *folded: it decodes with some key matched to its field only case-insensitively (the checks here read exact keys:
// such resources are not restated)
std::string typed_decode_error(const oj::VP& resource, const std::string& kind, bool* folded = nullptr);

}  // namespace orc
