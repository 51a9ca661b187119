// PodSecurity failure details on the host: RuleResponse.Message and RuleResponse.PodSecurityChecks of a failing
// podSecurity pair (pkg/engine/validation.go:550-564, pss.FormatChecksPrint pkg/pss/evaluate.go:160-166), rendered
// from the device's failing (check, version) slot mask and the resource's node table.
//
// The ForbiddenReason / ForbiddenDetail texts restate the default checks of k8s.io/pod-security-admission v0.26.1
// (policy/check_*.go; the module is not vendored under the reference): pinned by the kuttl report message
// (test/conformance/kuttl/reports/background/test-report-background-mode/report-assert.yaml), the other texts are
// parity unpinned. Rules with exclusions are not rendered here: exemptKyvernoExclusion rebuilds the check list from a
// Go map (evaluate.go:39-60), so the reference's order is nondeterministic.
#include <algorithm>
#include <array>
#include <set>

#include "kyv_host.h"

namespace kyv {

namespace {

// slot order of kyv_pss.h PssSlot = DefaultChecks() order (check files sorted by name), versions ascending
struct SlotInfo { const char* id; int check; };
const SlotInfo kSlots[] = {
    {"allowPrivilegeEscalation", 0}, {"allowPrivilegeEscalation", 0}, {"appArmorProfile", 1},
    {"capabilities_baseline", 2}, {"capabilities_restricted", 3}, {"capabilities_restricted", 3},
    {"hostNamespaces", 4}, {"hostPathVolumes", 5}, {"hostPorts", 6}, {"privileged", 7}, {"procMount", 8},
    {"restrictedVolumes", 9}, {"runAsNonRoot", 10}, {"runAsUser", 11}, {"seLinuxOptions", 12},
    {"seccompProfile_baseline", 13}, {"seccompProfile_baseline", 14}, {"seccompProfile_restricted", 15},
    {"seccompProfile_restricted", 15}, {"sysctls", 16}, {"windowsHostProcess", 17}};
constexpr int kNumSlots = (int)(sizeof(kSlots) / sizeof(kSlots[0]));

struct Tree {  // read-only view of one resource's nodes
  const Batch& b;
  const Node* R;
  const std::string& s(uint32_t sid) const { return b.dict.strs[sid]; }
  uint32_t get(uint32_t m, const char* key) const {
    if (m == NONE || node_type(R[m]) != N_MAP) return NONE;
    for (uint32_t i = R[m].a; i < R[m].a + R[m].b; i++)
      if (s(node_key(R[i])) == key) return node_type(R[i]) == N_NULL ? NONE : i;
    return NONE;
  }
  uint32_t type(uint32_t n) const { return n == NONE ? (uint32_t)N_NULL : node_type(R[n]); }
  std::string str(uint32_t n) const { return type(n) == N_STR ? s(R[n].a) : std::string(); }
  int pbool(uint32_t n) const { return type(n) == N_TRUE ? 1 : type(n) == N_FALSE ? 0 : -1; }
  bool i64(uint32_t n, int64_t* v) const {
    if (type(n) != N_INT) return false;
    *v = (int64_t)(((uint64_t)R[n].b << 32) | R[n].a);
    return true;
  }
  template <class F>
  void each(uint32_t arr, F f) const {
    if (type(arr) != N_ARR) return;
    for (uint32_t i = R[arr].a; i < R[arr].a + R[arr].b; i++) f(i);
  }
};

struct Ctr { std::string name, image; uint32_t node; uint32_t sc; };

std::string quote_list(const std::vector<std::string>& v) {  // policy/helpers.go joinQuote
  if (v.empty()) return "";
  std::string s = "\"";
  for (size_t i = 0; i < v.size(); i++) s += (i ? "\", \"" : "") + v[i];
  return s + "\"";
}
std::string join(const std::vector<std::string>& v, const char* sep) {
  std::string s;
  for (size_t i = 0; i < v.size(); i++) s += (i ? sep : "") + v[i];
  return s;
}
const char* plural(const char* one, const char* many, size_t n) { return n == 1 ? one : many; }
std::vector<std::string> sorted(const std::set<std::string>& x) { return {x.begin(), x.end()}; }
// strconv.Quote for the printable-ASCII strings this renderer accepts (others make the message unrenderable)
bool go_quote(const std::string& v, std::string* out) {
  std::string q = "\"";
  for (unsigned char c : v) {
    if (c < 0x20 || c >= 0x7F) return false;
    if (c == '"' || c == '\\') q += '\\';
    q += (char)c;
  }
  *out = q + "\"";
  return true;
}

struct Pod {
  const Tree& t;
  uint32_t meta, spec, psc;
  std::vector<Ctr> ctrs;  // init, regular, ephemeral (visitContainers order)
  bool windows = false;
};

struct Result { std::string reason, detail; };

std::string containers(const std::vector<std::string>& names) {
  return std::string(plural("container", "containers", names.size())) + " " + quote_list(names);
}

bool render_check(const Pod& p, int check, Result* r) {
  const Tree& t = p.t;
  switch (check) {
    case 0: {  // check_allowPrivilegeEscalation.go
      std::vector<std::string> bad;
      for (auto& c : p.ctrs) if (c.sc == NONE || t.pbool(t.get(c.sc, "allowPrivilegeEscalation")) != 0) bad.push_back(c.name);
      *r = {"allowPrivilegeEscalation != false", containers(bad) + " must set securityContext.allowPrivilegeEscalation=false"};
      return !bad.empty();
    }
    case 1: {  // check_appArmorProfile.go
      std::vector<std::string> bad;
      uint32_t ann = t.get(p.meta, "annotations");
      if (t.type(ann) == N_MAP)
        for (uint32_t i = t.R[ann].a; i < t.R[ann].a + t.R[ann].b; i++) {
          const std::string& k = t.s(node_key(t.R[i]));
          const std::string v = t.str(i);
          static const std::string pre = "container.apparmor.security.beta.kubernetes.io/";
          if (k.compare(0, pre.size(), pre) != 0 || v == "runtime/default" || v.compare(0, 10, "localhost/") == 0) continue;
          std::string q;
          if (!go_quote(v, &q)) return false;
          bad.push_back(k + "=" + q);
        }
      std::sort(bad.begin(), bad.end());
      *r = {plural("forbidden AppArmor profile", "forbidden AppArmor profiles", bad.size()), join(bad, ", ")};
      return !bad.empty();
    }
    case 2: {  // check_capabilities_baseline.go
      static const std::set<std::string> ok = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID", "KILL", "MKNOD",
                                               "NET_BIND_SERVICE", "SETFCAP", "SETGID", "SETPCAP", "SETUID", "SYS_CHROOT"};
      std::vector<std::string> bad;
      std::set<std::string> caps;
      for (auto& c : p.ctrs) {
        uint32_t cp = t.get(c.sc, "capabilities");
        if (cp == NONE) continue;
        bool valid = true;
        t.each(t.get(cp, "add"), [&](uint32_t a) { if (!ok.count(t.str(a))) { valid = false; caps.insert(t.str(a)); } });
        if (!valid) bad.push_back(c.name);
      }
      *r = {"non-default capabilities",
            containers(bad) + " must not include " + quote_list(sorted(caps)) + " in securityContext.capabilities.add"};
      return !bad.empty();
    }
    case 3: {  // check_capabilities_restricted.go
      std::vector<std::string> nodrop, adds;
      std::set<std::string> forbidden;
      for (auto& c : p.ctrs) {
        uint32_t cp = t.get(c.sc, "capabilities");
        if (cp == NONE) { nodrop.push_back(c.name); continue; }
        bool all = false, extra = false;
        t.each(t.get(cp, "drop"), [&](uint32_t d) { all = all || t.str(d) == "ALL"; });
        t.each(t.get(cp, "add"), [&](uint32_t a) { if (t.str(a) != "NET_BIND_SERVICE") { extra = true; forbidden.insert(t.str(a)); } });
        if (!all) nodrop.push_back(c.name);
        if (extra) adds.push_back(c.name);
      }
      std::vector<std::string> d;
      if (!nodrop.empty()) d.push_back(containers(nodrop) + " must set securityContext.capabilities.drop=[\"ALL\"]");
      if (!adds.empty())
        d.push_back(containers(adds) + " must not include " + quote_list(sorted(forbidden)) + " in securityContext.capabilities.add");
      *r = {"unrestricted capabilities", join(d, "; ")};
      return !d.empty();
    }
    case 4: {  // check_hostNamespaces.go
      std::vector<std::string> h;
      if (t.pbool(t.get(p.spec, "hostNetwork")) == 1) h.push_back("hostNetwork=true");
      if (t.pbool(t.get(p.spec, "hostPID")) == 1) h.push_back("hostPID=true");
      if (t.pbool(t.get(p.spec, "hostIPC")) == 1) h.push_back("hostIPC=true");
      *r = {"host namespaces", join(h, ", ")};
      return !h.empty();
    }
    case 5: {  // check_hostPathVolumes.go
      std::vector<std::string> h;
      t.each(t.get(p.spec, "volumes"), [&](uint32_t v) { if (t.get(v, "hostPath") != NONE) h.push_back(t.str(t.get(v, "name"))); });
      *r = {"hostPath volumes", std::string(plural("volume", "volumes", h.size())) + " " + quote_list(h)};
      return !h.empty();
    }
    case 6: {  // check_hostPorts.go
      std::vector<std::string> bad;
      std::set<int64_t> ports;
      for (auto& c : p.ctrs) {
        bool valid = true;
        t.each(t.get(c.node, "ports"), [&](uint32_t pt) {
          int64_t hp = 0;
          if (t.i64(t.get(pt, "hostPort"), &hp) && hp != 0) { valid = false; ports.insert(hp); }
        });
        if (!valid) bad.push_back(c.name);
      }
      std::vector<std::string> ps;  // sets.String of the decimal forms: sorted as strings
      std::set<std::string> pstr;
      for (auto x : ports) pstr.insert(std::to_string(x));
      ps.assign(pstr.begin(), pstr.end());
      *r = {"hostPort", containers(bad) + " " + plural("uses", "use", bad.size()) + " " +
                            plural("hostPort", "hostPorts", ps.size()) + " " + join(ps, ", ")};
      return !bad.empty();
    }
    case 7: {  // check_privileged.go
      std::vector<std::string> bad;
      for (auto& c : p.ctrs) if (t.pbool(t.get(c.sc, "privileged")) == 1) bad.push_back(c.name);
      *r = {"privileged", containers(bad) + " must not set securityContext.privileged=true"};
      return !bad.empty();
    }
    case 8: {  // check_procMount.go
      std::vector<std::string> bad;
      std::set<std::string> types;
      for (auto& c : p.ctrs) {
        uint32_t pm = t.get(c.sc, "procMount");
        if (pm == NONE || t.str(pm) == "Default") continue;
        bad.push_back(c.name);
        types.insert(t.str(pm));
      }
      *r = {"procMount", containers(bad) + " must not set securityContext.procMount to " + quote_list(sorted(types))};
      return !bad.empty();
    }
    case 9: {  // check_restrictedVolumes.go
      static const char* allowed[] = {"configMap", "csi", "downwardAPI", "emptyDir", "ephemeral", "persistentVolumeClaim",
                                      "projected", "secret"};
      static const char* named[] = {"hostPath", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "nfs", "iscsi",
                                    "glusterfs", "rbd", "flexVolume", "cinder", "cephfs", "flocker", "fc", "azureFile",
                                    "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk", "portworxVolume",
                                    "scaleIO", "storageos"};
      std::vector<std::string> bad;
      std::set<std::string> types;
      t.each(t.get(p.spec, "volumes"), [&](uint32_t v) {
        for (const char* a : allowed) if (t.get(v, a) != NONE) return;
        bad.push_back(t.str(t.get(v, "name")));
        std::string ty = "unknown";
        for (const char* n : named) if (t.get(v, n) != NONE) { ty = n; break; }
        types.insert(ty);
      });
      *r = {"restricted volume types", std::string(plural("volume", "volumes", bad.size())) + " " + quote_list(bad) + " " +
                                           plural("uses", "use", bad.size()) + " " +
                                           plural("restricted volume type", "restricted volume types", types.size()) + " " +
                                           quote_list(sorted(types))};
      return !bad.empty();
    }
    case 10: {  // check_runAsNonRoot.go
      std::vector<std::string> who, expl, impl;
      const int pod = t.pbool(t.get(p.psc, "runAsNonRoot"));
      if (pod == 0) who.push_back("pod");
      for (auto& c : p.ctrs) {
        const int v = t.pbool(t.get(c.sc, "runAsNonRoot"));
        if (v == 0) expl.push_back(c.name);
        else if (v == -1 && pod != 1) impl.push_back(c.name);
      }
      if (!expl.empty()) who.push_back(containers(expl));
      if (!who.empty()) { *r = {"runAsNonRoot != true", join(who, " and ") + " must not set securityContext.runAsNonRoot=false"}; return true; }
      *r = {"runAsNonRoot != true", "pod or " + containers(impl) + " must set securityContext.runAsNonRoot=true"};
      return !impl.empty();
    }
    case 11: {  // check_runAsUser.go
      std::vector<std::string> who, expl;
      int64_t u;
      if (t.i64(t.get(p.psc, "runAsUser"), &u) && u == 0) who.push_back("pod");
      for (auto& c : p.ctrs) if (t.i64(t.get(c.sc, "runAsUser"), &u) && u == 0) expl.push_back(c.name);
      if (!expl.empty()) who.push_back(containers(expl));
      *r = {"runAsUser=0", join(who, " and ") + " must not set runAsUser=0"};
      return !who.empty();
    }
    case 12: {  // check_seLinuxOptions.go
      static const std::set<std::string> okt = {"", "container_t", "container_init_t", "container_kvm_t"};
      std::vector<std::string> who, bad;
      std::set<std::string> types;
      bool user = false, role = false;
      auto valid = [&](uint32_t o) {
        bool v = true;
        const std::string ty = t.str(t.get(o, "type"));
        if (!okt.count(ty)) { v = false; types.insert(ty); }
        if (!t.str(t.get(o, "user")).empty()) { v = false; user = true; }
        if (!t.str(t.get(o, "role")).empty()) { v = false; role = true; }
        return v;
      };
      uint32_t ps = t.get(p.psc, "seLinuxOptions");
      if (ps != NONE && !valid(ps)) who.push_back("pod");
      for (auto& c : p.ctrs) {
        uint32_t cs = t.get(c.sc, "seLinuxOptions");
        if (cs != NONE && !valid(cs)) bad.push_back(c.name);
      }
      if (!bad.empty()) who.push_back(containers(bad));
      std::vector<std::string> d;
      if (!types.empty()) d.push_back(std::string(plural("type", "types", types.size())) + " " + quote_list(sorted(types)));
      if (user) d.push_back("user may not be set");
      if (role) d.push_back("role may not be set");
      *r = {"seLinuxOptions", join(who, " and ") + " set forbidden securityContext.seLinuxOptions: " + join(d, "; ")};
      return !who.empty();
    }
    case 13: {  // check_seccompProfile_baseline.go v1.0 (annotations)
      std::set<std::string> bad;
      uint32_t ann = t.get(p.meta, "annotations");
      auto look = [&](const std::string& key) {
        uint32_t a = t.get(ann, key.c_str());
        if (a != NONE && t.str(a) == "unconfined") bad.insert(key + "=\"unconfined\"");
      };
      look("seccomp.security.alpha.kubernetes.io/pod");
      for (auto& c : p.ctrs) look("container.seccomp.security.alpha.kubernetes.io/" + c.name);
      *r = {"seccompProfile", std::string("forbidden ") + plural("annotation", "annotations", bad.size()) + " " +
                                  join(sorted(bad), ", ")};
      return !bad.empty();
    }
    case 14: {  // check_seccompProfile_baseline.go v1.19
      std::vector<std::string> who, bad;
      std::set<std::string> vals;
      if (t.str(t.get(t.get(p.psc, "seccompProfile"), "type")) == "Unconfined" && t.get(p.psc, "seccompProfile") != NONE) {
        who.push_back("pod");
        vals.insert("Unconfined");
      }
      for (auto& c : p.ctrs) {
        uint32_t sp = t.get(c.sc, "seccompProfile");
        if (sp != NONE && t.str(t.get(sp, "type")) == "Unconfined") { bad.push_back(c.name); vals.insert("Unconfined"); }
      }
      if (!bad.empty()) who.push_back(containers(bad));
      *r = {"seccompProfile", join(who, " and ") + " must not set securityContext.seccompProfile.type to " + quote_list(sorted(vals))};
      return !who.empty();
    }
    case 15: {  // check_seccompProfile_restricted.go
      auto ok = [](const std::string& x) { return x == "Localhost" || x == "RuntimeDefault"; };
      std::vector<std::string> who, expl, impl;
      std::set<std::string> vals;
      bool podSet = false;
      uint32_t ps = t.get(p.psc, "seccompProfile");
      if (ps != NONE) {
        const std::string ty = t.str(t.get(ps, "type"));
        if (!ok(ty)) { who.push_back("pod"); vals.insert(ty); } else podSet = true;
      }
      for (auto& c : p.ctrs) {
        uint32_t sp = t.get(c.sc, "seccompProfile");
        if (sp != NONE) {
          const std::string ty = t.str(t.get(sp, "type"));
          if (!ok(ty)) { expl.push_back(c.name); vals.insert(ty); }
        } else if (!podSet) {
          impl.push_back(c.name);
        }
      }
      if (!expl.empty()) who.push_back(containers(expl));
      if (!who.empty()) {
        *r = {"seccompProfile", join(who, " and ") + " must not set securityContext.seccompProfile.type to " + quote_list(sorted(vals))};
        return true;
      }
      *r = {"seccompProfile", "pod or " + containers(impl) +
                                  " must set securityContext.seccompProfile.type to \"RuntimeDefault\" or \"Localhost\""};
      return !impl.empty();
    }
    case 16: {  // check_sysctls.go
      static const std::set<std::string> ok = {"kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range",
                                               "net.ipv4.tcp_syncookies", "net.ipv4.ping_group_range",
                                               "net.ipv4.ip_unprivileged_port_start"};
      std::vector<std::string> bad;
      t.each(t.get(p.psc, "sysctls"), [&](uint32_t s) {
        const std::string n = t.str(t.get(s, "name"));
        if (!ok.count(n)) bad.push_back(n);
      });
      *r = {"forbidden sysctls", join(bad, ", ")};
      return !bad.empty();
    }
    case 17: {  // check_windowsHostProcess.go
      std::vector<std::string> who, bad;
      for (auto& c : p.ctrs) if (t.pbool(t.get(t.get(c.sc, "windowsOptions"), "hostProcess")) == 1) bad.push_back(c.name);
      if (t.pbool(t.get(t.get(p.psc, "windowsOptions"), "hostProcess")) == 1) who.push_back("pod");
      if (!bad.empty()) who.push_back(containers(bad));
      *r = {"hostProcess", join(who, " and ") + " must not set securityContext.windowsOptions.hostProcess=true"};
      return !who.empty();
    }
  }
  return false;
}

}  // namespace

// One failing podSecurity pair -> (check id, reason, detail) per failing slot in DefaultChecks() order; false when the
// pair is not renderable here (exclusions, strings outside printable ASCII in quoted values, non-pod kinds)
bool pss_checks_render(const Ruleset& rs, const Batch& b, uint32_t pos, uint32_t rule, uint32_t mask,
                       std::vector<std::array<std::string, 3>>* out) {
  const RuleDesc& rd = rs.rules[rule];
  if (rd.kind != RK_PSS || rs.pss[rd.root].nexcl) return false;
  const ResHeader& h = b.hdr[pos];
  Tree t{b, b.nodes.data() + h.root};
  const std::string kind = b.dict.strs[h.kind];
  uint32_t meta = NONE, spec = NONE;
  if (kind == "Pod") {
    meta = t.get(0, "metadata");
    spec = t.get(0, "spec");
  } else if (kind == "CronJob") {
    uint32_t jt = t.get(t.get(0, "spec"), "jobTemplate");
    meta = t.get(jt, "metadata");
    spec = t.get(t.get(t.get(jt, "spec"), "template"), "spec");
  } else if (kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
             kind == "ReplicaSet" || kind == "ReplicationController") {
    uint32_t tpl = t.get(t.get(0, "spec"), "template");
    meta = t.get(tpl, "metadata");
    spec = t.get(tpl, "spec");
  } else {
    return false;
  }
  Pod p{t, meta, spec, t.get(spec, "securityContext"), {}, false};
  for (const char* list : {"initContainers", "containers", "ephemeralContainers"})
    t.each(t.get(spec, list), [&](uint32_t c) {
      p.ctrs.push_back(Ctr{t.str(t.get(c, "name")), t.str(t.get(c, "image")), c, t.get(c, "securityContext")});
    });
  out->clear();
  for (int s = 0; s < kNumSlots; s++) {
    if (!((mask >> s) & 1u)) continue;
    Result r;
    if (!render_check(p, kSlots[s].check, &r)) return false;  // mask and restated check disagree: do not guess
    out->push_back({kSlots[s].id, r.reason, r.detail});
  }
  return !out->empty();
}

}  // namespace kyv
