// ORACLE — test infrastructure only (see ojson.h header).
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ojson.h"
#include "opss.h"

namespace orc {

struct RuleResult {
  std::string name;
  std::string status;  // pass fail skip error | unsupported (needs JMESPath/vars/deny/foreach) | panic | none
  std::string message;
  std::string path;    // failing path for single-pattern fails
  std::vector<std::string> branch_paths;  // anyPattern per-branch paths
  std::vector<PSSResult> pss_checks;
  bool nondeterministic = false;  // verdict depends on Go map order in the reference
  bool message_unpinned = false;  // message text order/content not pinned (PSS excludes / decode errors)
  bool deny_message = false;      // deny failure message rendered by render_message (variables resolved)
};

struct PolicyResult {
  std::string name;
  bool namespace_skipped = false;
  bool truncated_unknown = false;
  std::vector<RuleResult> rules;
};

std::vector<oj::VP> compute_rules(const oj::VP& policy);
bool matches_resource_description(const oj::VP& rule, const oj::VP& resource, const std::map<std::string, std::string>& nsl,
                                  bool* nd);
RuleResult validate_rule(const oj::VP& rule, const oj::VP& resource);
// PolicyException documents the following runs check (hasPolicyExceptions); set before the run's threads start
void set_exceptions(const std::vector<oj::VP>& ex);
std::string nested_string(const oj::VP& obj, std::initializer_list<const char*> path);
bool has_nonempty(const oj::VP& o, const char* k);
PolicyResult validate_policy(const oj::VP& policy, const oj::VP& resource, const std::map<std::string, std::string>& nsLabels);
PolicyResult validate_policy_rules(const oj::VP& policy, const std::vector<oj::VP>& rules, const oj::VP& resource,
                                   const std::map<std::string, std::string>& nsLabels);
std::string rule_unsupported_reason(const oj::VP& rule);
void get_kind_from_gvk(const std::string& str, std::string& gv, std::string& kind);

}  // namespace orc
