// ORACLE — test infrastructure only (see ojson.h header).
//
// Restatement of pkg/pss/evaluate.go (EvaluatePod :83, evaluatePSS :16, exemptKyvernoExclusion :39,
// GetPodWithMatchingContainers :112, FormatChecksPrint :160) and of the default checks of
// k8s.io/pod-security-admission v0.26.1 policy.DefaultChecks() — that module is NOT vendored under
// /root/reference; its published algorithm is restated here and pinned by the 128 verdict cases of
// pkg/pss/evaluate_test.go plus the one message in
// test/conformance/kuttl/reports/background/test-report-background-mode/report-assert.yaml.
//
// The typed decode (validation.go:481-532 getSpec -> json.Unmarshal into corev1.Pod / appsv1.Deployment /
// batchv1.CronJob) is modelled for the fields the checks read: a JSON type mismatch on those fields is a
// decode error (-> rule error).
#include "opss.h"

#include <algorithm>
#include <set>

#include "goutil.h"

namespace orc {
using oj::T;
using oj::VP;

namespace {

struct DecodeError { std::string msg; };

bool isnil(const VP& v) { return !v || v->t == T::Null; }

// typed accessors (json.Unmarshal semantics: null -> zero value; wrong JSON type -> error)
const VP& want_obj(const VP& v, const char* what) {
  if (!isnil(v) && v->t != T::Obj) throw DecodeError{std::string("json: cannot unmarshal into ") + what};
  return v;
}
std::string want_str(const VP& v, const char* what) {
  if (isnil(v)) return "";
  if (v->t != T::Str) throw DecodeError{std::string("json: cannot unmarshal into string field ") + what};
  return v->s;
}
// *bool
int want_pbool(const VP& v, const char* what) {  // -1 nil, 0 false, 1 true
  if (isnil(v)) return -1;
  if (v->t != T::Bool) throw DecodeError{std::string("json: cannot unmarshal into bool field ") + what};
  return v->b ? 1 : 0;
}
bool want_bool(const VP& v, const char* what) { return want_pbool(v, what) == 1; }
bool want_int(const VP& v, const char* what, int64_t lo, int64_t hi, int64_t& out) {  // false if nil
  if (isnil(v)) return false;
  if (v->t != T::Int || v->i < lo || v->i > hi) throw DecodeError{std::string("json: cannot unmarshal into int field ") + what};
  out = v->i;
  return true;
}
std::vector<VP> want_arr(const VP& v, const char* what) {
  if (isnil(v)) return {};
  if (v->t != T::Arr) throw DecodeError{std::string("json: cannot unmarshal into slice ") + what};
  return v->a;
}

struct SELinux { bool set = false; std::string user, role, type, level; };
struct Seccomp { bool set = false; std::string type; };
struct WinOpts { bool set = false; int hostProcess = -1; };
struct SecCtx {
  bool set = false;
  int privileged = -1, ape = -1, runAsNonRoot = -1;
  bool hasRunAsUser = false; int64_t runAsUser = 0;
  SELinux selinux; Seccomp seccomp; WinOpts win;
  bool capsSet = false; std::vector<std::string> add, drop;
  bool procMountSet = false; std::string procMount;
};
struct Container { std::string name, image; std::vector<int64_t> hostPorts; SecCtx sc; };
struct PodSC {
  bool set = false; int runAsNonRoot = -1; bool hasRunAsUser = false; int64_t runAsUser = 0;
  SELinux selinux; Seccomp seccomp; WinOpts win; std::vector<std::string> sysctls;
};
struct Volume { std::string name; std::set<std::string> sources; };  // non-nil typed VolumeSource members
struct Pod {
  std::string name, ns;
  std::map<std::string, std::string> annotations;
  bool hostNetwork = false, hostPID = false, hostIPC = false;
  PodSC sc;
  std::vector<Container> containers, init, ephemeral;
  std::vector<Volume> volumes;
  std::string osName;
};

SELinux dec_selinux(const VP& v) {
  SELinux s;
  want_obj(v, "SELinuxOptions");
  if (isnil(v)) return s;
  s.set = true;
  s.user = want_str(v->get("user"), "user");
  s.role = want_str(v->get("role"), "role");
  s.type = want_str(v->get("type"), "type");
  s.level = want_str(v->get("level"), "level");
  return s;
}
Seccomp dec_seccomp(const VP& v) {
  Seccomp s;
  want_obj(v, "SeccompProfile");
  if (isnil(v)) return s;
  s.set = true;
  s.type = want_str(v->get("type"), "type");
  want_str(v->get("localhostProfile"), "localhostProfile");
  return s;
}
WinOpts dec_win(const VP& v) {
  WinOpts w;
  want_obj(v, "WindowsSecurityContextOptions");
  if (isnil(v)) return w;
  w.set = true;
  w.hostProcess = want_pbool(v->get("hostProcess"), "hostProcess");
  want_str(v->get("gmsaCredentialSpecName"), "gmsaCredentialSpecName");
  want_str(v->get("gmsaCredentialSpec"), "gmsaCredentialSpec");
  want_str(v->get("runAsUserName"), "runAsUserName");
  return w;
}

Container dec_container(const VP& v) {
  Container c;
  want_obj(v, "Container");
  if (isnil(v)) return c;
  c.name = want_str(v->get("name"), "name");
  c.image = want_str(v->get("image"), "image");
  for (auto& p : want_arr(v->get("ports"), "ports")) {
    want_obj(p, "ContainerPort");
    int64_t hp = 0;
    if (!isnil(p)) {
      want_int(p->get("hostPort"), "hostPort", INT32_MIN, INT32_MAX, hp);
      int64_t cp;
      want_int(p->get("containerPort"), "containerPort", INT32_MIN, INT32_MAX, cp);
      want_str(p->get("name"), "name");
      want_str(p->get("protocol"), "protocol");
      want_str(p->get("hostIP"), "hostIP");
    }
    c.hostPorts.push_back(hp);
  }
  // commonly set fields beyond what the checks read (env, command / args, workingDir, imagePullPolicy)
  for (auto& e : want_arr(v->get("env"), "env")) {
    want_obj(e, "EnvVar");
    if (isnil(e)) continue;
    want_str(e->get("name"), "name");
    want_str(e->get("value"), "value");
    want_obj(e->get("valueFrom"), "EnvVarSource");
  }
  for (const char* k : {"command", "args"})
    for (auto& s : want_arr(v->get(k), k)) want_str(s, k);
  want_str(v->get("workingDir"), "workingDir");
  want_str(v->get("imagePullPolicy"), "imagePullPolicy");
  VP sc = v->get("securityContext");
  want_obj(sc, "SecurityContext");
  if (!isnil(sc)) {
    c.sc.set = true;
    c.sc.privileged = want_pbool(sc->get("privileged"), "privileged");
    c.sc.ape = want_pbool(sc->get("allowPrivilegeEscalation"), "allowPrivilegeEscalation");
    c.sc.runAsNonRoot = want_pbool(sc->get("runAsNonRoot"), "runAsNonRoot");
    want_pbool(sc->get("readOnlyRootFilesystem"), "readOnlyRootFilesystem");
    c.sc.hasRunAsUser = want_int(sc->get("runAsUser"), "runAsUser", INT64_MIN, INT64_MAX, c.sc.runAsUser);
    int64_t g;
    want_int(sc->get("runAsGroup"), "runAsGroup", INT64_MIN, INT64_MAX, g);
    c.sc.selinux = dec_selinux(sc->get("seLinuxOptions"));
    c.sc.seccomp = dec_seccomp(sc->get("seccompProfile"));
    c.sc.win = dec_win(sc->get("windowsOptions"));
    VP caps = sc->get("capabilities");
    want_obj(caps, "Capabilities");
    if (!isnil(caps)) {
      c.sc.capsSet = true;
      for (auto& a : want_arr(caps->get("add"), "add")) c.sc.add.push_back(want_str(a, "add"));
      for (auto& d : want_arr(caps->get("drop"), "drop")) c.sc.drop.push_back(want_str(d, "drop"));
    }
    VP pm = sc->get("procMount");
    if (!isnil(pm)) { c.sc.procMountSet = true; c.sc.procMount = want_str(pm, "procMount"); }
  }
  return c;
}

static const char* kVolumeSources[] = {
    "hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "secret", "nfs", "iscsi",
    "glusterfs", "persistentVolumeClaim", "rbd", "flexVolume", "cinder", "cephfs", "flocker", "downwardAPI", "fc",
    "azureFile", "configMap", "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk", "projected",
    "portworxVolume", "scaleIO", "storageos", "csi", "ephemeral"};

// podSpec + metadata
Pod dec_pod(const VP& meta, const VP& spec) {
  Pod p;
  want_obj(meta, "ObjectMeta");
  if (!isnil(meta)) {
    p.name = want_str(meta->get("name"), "name");
    p.ns = want_str(meta->get("namespace"), "namespace");
    VP ann = meta->get("annotations");
    want_obj(ann, "annotations");
    if (!isnil(ann))
      for (auto& kv : ann->o) {
        if (isnil(kv.second)) { p.annotations[kv.first] = ""; continue; }
        p.annotations[kv.first] = want_str(kv.second, "annotations");
      }
    VP lab = meta->get("labels");
    want_obj(lab, "labels");
    if (!isnil(lab)) for (auto& kv : lab->o) want_str(kv.second, "labels");
  }
  want_obj(spec, "PodSpec");
  if (isnil(spec)) return p;
  p.hostNetwork = want_bool(spec->get("hostNetwork"), "hostNetwork");
  p.hostPID = want_bool(spec->get("hostPID"), "hostPID");
  p.hostIPC = want_bool(spec->get("hostIPC"), "hostIPC");
  VP sc = spec->get("securityContext");
  want_obj(sc, "PodSecurityContext");
  if (!isnil(sc)) {
    p.sc.set = true;
    p.sc.runAsNonRoot = want_pbool(sc->get("runAsNonRoot"), "runAsNonRoot");
    p.sc.hasRunAsUser = want_int(sc->get("runAsUser"), "runAsUser", INT64_MIN, INT64_MAX, p.sc.runAsUser);
    int64_t g;
    want_int(sc->get("runAsGroup"), "runAsGroup", INT64_MIN, INT64_MAX, g);
    want_int(sc->get("fsGroup"), "fsGroup", INT64_MIN, INT64_MAX, g);
    for (auto& x : want_arr(sc->get("supplementalGroups"), "supplementalGroups")) {
      int64_t y;
      if (isnil(x)) continue;
      want_int(x, "supplementalGroups", INT64_MIN, INT64_MAX, y);
    }
    p.sc.selinux = dec_selinux(sc->get("seLinuxOptions"));
    p.sc.seccomp = dec_seccomp(sc->get("seccompProfile"));
    p.sc.win = dec_win(sc->get("windowsOptions"));
    for (auto& s : want_arr(sc->get("sysctls"), "sysctls")) {
      want_obj(s, "Sysctl");
      if (isnil(s)) { p.sc.sysctls.push_back(""); continue; }
      p.sc.sysctls.push_back(want_str(s->get("name"), "name"));
      want_str(s->get("value"), "value");
    }
  }
  for (auto& c : want_arr(spec->get("containers"), "containers")) p.containers.push_back(dec_container(c));
  for (auto& c : want_arr(spec->get("initContainers"), "initContainers")) p.init.push_back(dec_container(c));
  for (auto& c : want_arr(spec->get("ephemeralContainers"), "ephemeralContainers")) p.ephemeral.push_back(dec_container(c));
  for (auto& v : want_arr(spec->get("volumes"), "volumes")) {
    want_obj(v, "Volume");
    Volume vol;
    if (!isnil(v)) {
      vol.name = want_str(v->get("name"), "name");
      for (const char* src : kVolumeSources) {
        VP sv = v->get(src);
        want_obj(sv, src);
        if (!isnil(sv)) vol.sources.insert(src);
      }
    }
    p.volumes.push_back(vol);
  }
  VP os = spec->get("os");
  want_obj(os, "PodOS");
  if (!isnil(os)) p.osName = want_str(os->get("name"), "name");
  // commonly set fields beyond what the checks read
  VP nsel = spec->get("nodeSelector");
  want_obj(nsel, "nodeSelector");
  if (!isnil(nsel)) for (auto& kv : nsel->o) want_str(kv.second, "nodeSelector");
  want_str(spec->get("serviceAccountName"), "serviceAccountName");
  want_str(spec->get("restartPolicy"), "restartPolicy");
  int64_t t;
  want_int(spec->get("terminationGracePeriodSeconds"), "terminationGracePeriodSeconds", INT64_MIN, INT64_MAX, t);
  want_int(spec->get("activeDeadlineSeconds"), "activeDeadlineSeconds", INT64_MIN, INT64_MAX, t);
  return p;
}

// ---- pod-security-admission helpers (policy/helpers.go) ----
std::string join_quote(const std::vector<std::string>& items) {
  if (items.empty()) return "";
  std::string s = "\"";
  for (size_t i = 0; i < items.size(); i++) { if (i) s += "\", \""; s += items[i]; }
  return s + "\"";
}
const char* pluralize(const char* a, const char* b, size_t n) { return n == 1 ? a : b; }
std::string join(const std::vector<std::string>& v, const std::string& sep) {
  std::string s;
  for (size_t i = 0; i < v.size(); i++) { if (i) s += sep; s += v[i]; }
  return s;
}
template <class F>
void visit_containers(const Pod& p, F f) {
  for (auto& c : p.init) f(c);
  for (auto& c : p.containers) f(c);
  for (auto& c : p.ephemeral) f(c);
}
std::vector<std::string> sorted(const std::set<std::string>& s) { return std::vector<std::string>(s.begin(), s.end()); }

using CR = CheckResult;
CR allowed() { return CR{true, "", ""}; }

CR allowPrivilegeEscalation_1_8(const Pod& p) {
  std::vector<std::string> bad;
  visit_containers(p, [&](const Container& c) { if (!c.sc.set || c.sc.ape != 0) bad.push_back(c.name); });
  if (!bad.empty())
    return CR{false, "allowPrivilegeEscalation != false",
              std::string(pluralize("container", "containers", bad.size())) + " " + join_quote(bad) +
                  " must set securityContext.allowPrivilegeEscalation=false"};
  return allowed();
}
bool windows(const Pod& p) { return p.osName == "windows"; }
CR allowPrivilegeEscalation_1_25(const Pod& p) { return windows(p) ? allowed() : allowPrivilegeEscalation_1_8(p); }

CR appArmorProfile_1_0(const Pod& p) {
  std::vector<std::string> bad;
  for (auto& kv : p.annotations) {
    const std::string pre = "container.apparmor.security.beta.kubernetes.io/";
    if (kv.first.compare(0, pre.size(), pre) == 0 && kv.second != "runtime/default" && kv.second.compare(0, 10, "localhost/") != 0)
      bad.push_back(kv.first + "=" + gou::go_quote(kv.second));
  }
  if (!bad.empty()) {
    std::sort(bad.begin(), bad.end());
    return CR{false, pluralize("forbidden AppArmor profile", "forbidden AppArmor profiles", bad.size()), join(bad, ", ")};
  }
  return allowed();
}

CR capabilitiesBaseline_1_0(const Pod& p) {
  static const std::set<std::string> ok = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID", "KILL", "MKNOD",
                                           "NET_BIND_SERVICE", "SETFCAP", "SETGID", "SETPCAP", "SETUID", "SYS_CHROOT"};
  std::vector<std::string> bad;
  std::set<std::string> caps;
  visit_containers(p, [&](const Container& c) {
    if (c.sc.set && c.sc.capsSet) {
      bool valid = true;
      for (auto& a : c.sc.add) if (!ok.count(a)) { valid = false; caps.insert(a); }
      if (!valid) bad.push_back(c.name);
    }
  });
  if (!bad.empty())
    return CR{false, "non-default capabilities",
              std::string(pluralize("container", "containers", bad.size())) + " " + join_quote(bad) + " must not include " +
                  join_quote(sorted(caps)) + " in securityContext.capabilities.add"};
  return allowed();
}

CR capabilitiesRestricted_1_22(const Pod& p) {
  std::vector<std::string> missing, adding;
  std::set<std::string> forb;
  visit_containers(p, [&](const Container& c) {
    if (!c.sc.set || !c.sc.capsSet) { missing.push_back(c.name); return; }
    bool all = false;
    for (auto& d : c.sc.drop) if (d == "ALL") { all = true; break; }
    if (!all) missing.push_back(c.name);
    bool af = false;
    for (auto& a : c.sc.add) if (a != "NET_BIND_SERVICE") { af = true; forb.insert(a); }
    if (af) adding.push_back(c.name);
  });
  std::vector<std::string> det;
  if (!missing.empty())
    det.push_back(std::string(pluralize("container", "containers", missing.size())) + " " + join_quote(missing) +
                  " must set securityContext.capabilities.drop=[\"ALL\"]");
  if (!adding.empty())
    det.push_back(std::string(pluralize("container", "containers", adding.size())) + " " + join_quote(adding) +
                  " must not include " + join_quote(sorted(forb)) + " in securityContext.capabilities.add");
  if (!det.empty()) return CR{false, "unrestricted capabilities", join(det, "; ")};
  return allowed();
}
CR capabilitiesRestricted_1_25(const Pod& p) { return windows(p) ? allowed() : capabilitiesRestricted_1_22(p); }

CR hostNamespaces_1_0(const Pod& p) {
  std::vector<std::string> h;
  if (p.hostNetwork) h.push_back("hostNetwork=true");
  if (p.hostPID) h.push_back("hostPID=true");
  if (p.hostIPC) h.push_back("hostIPC=true");
  if (!h.empty()) return CR{false, "host namespaces", join(h, ", ")};
  return allowed();
}

CR hostPathVolumes_1_0(const Pod& p) {
  std::vector<std::string> h;
  for (auto& v : p.volumes) if (v.sources.count("hostPath")) h.push_back(v.name);
  if (!h.empty()) return CR{false, "hostPath volumes", std::string(pluralize("volume", "volumes", h.size())) + " " + join_quote(h)};
  return allowed();
}

CR hostPorts_1_0(const Pod& p) {
  std::vector<std::string> bad;
  std::set<std::string> ports;
  visit_containers(p, [&](const Container& c) {
    bool valid = true;
    for (auto hp : c.hostPorts) if (hp != 0) { valid = false; ports.insert(std::to_string(hp)); }
    if (!valid) bad.push_back(c.name);
  });
  if (!bad.empty())
    return CR{false, "hostPort",
              std::string(pluralize("container", "containers", bad.size())) + " " + join_quote(bad) + " " +
                  pluralize("uses", "use", bad.size()) + " " + pluralize("hostPort", "hostPorts", ports.size()) + " " +
                  join(sorted(ports), ", ")};
  return allowed();
}

CR privileged_1_0(const Pod& p) {
  std::vector<std::string> bad;
  visit_containers(p, [&](const Container& c) { if (c.sc.set && c.sc.privileged == 1) bad.push_back(c.name); });
  if (!bad.empty())
    return CR{false, "privileged",
              std::string(pluralize("container", "containers", bad.size())) + " " + join_quote(bad) +
                  " must not set securityContext.privileged=true"};
  return allowed();
}

CR procMount_1_0(const Pod& p) {
  std::vector<std::string> bad;
  std::set<std::string> types;
  visit_containers(p, [&](const Container& c) {
    if (!c.sc.set || !c.sc.procMountSet) return;
    if (c.sc.procMount != "Default") { bad.push_back(c.name); types.insert(c.sc.procMount); }
  });
  if (!bad.empty())
    return CR{false, "procMount",
              std::string(pluralize("container", "containers", bad.size())) + " " + join_quote(bad) +
                  " must not set securityContext.procMount to " + join_quote(sorted(types))};
  return allowed();
}

CR restrictedVolumes_1_0(const Pod& p) {
  static const std::set<std::string> okv = {"configMap", "csi", "downwardAPI", "emptyDir", "ephemeral",
                                            "persistentVolumeClaim", "projected", "secret"};
  // restricted.go switch order for naming the forbidden source
  static const char* named[] = {"hostPath", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "nfs", "iscsi",
                                "glusterfs", "rbd", "flexVolume", "cinder", "cephfs", "flocker", "fc", "azureFile",
                                "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk", "portworxVolume",
                                "scaleIO", "storageos"};
  std::vector<std::string> bad;
  std::set<std::string> types;
  for (auto& v : p.volumes) {
    bool allowedSrc = false;
    for (auto& s : v.sources) if (okv.count(s)) allowedSrc = true;
    if (allowedSrc) continue;
    bad.push_back(v.name);
    std::string t = "unknown";
    for (const char* n : named) if (v.sources.count(n)) { t = n; break; }
    types.insert(t);
  }
  if (!bad.empty())
    return CR{false, "restricted volume types",
              std::string(pluralize("volume", "volumes", bad.size())) + " " + join_quote(bad) + " " +
                  pluralize("uses", "use", bad.size()) + " " +
                  pluralize("restricted volume type", "restricted volume types", types.size()) + " " +
                  join_quote(sorted(types))};
  return allowed();
}

CR runAsNonRoot_1_0(const Pod& p) {
  std::vector<std::string> setters, expl, impl;
  bool podOK = false;
  if (p.sc.set && p.sc.runAsNonRoot != -1) {
    if (p.sc.runAsNonRoot == 0) setters.push_back("pod");
    else podOK = true;
  }
  visit_containers(p, [&](const Container& c) {
    if (c.sc.set && c.sc.runAsNonRoot != -1) {
      if (c.sc.runAsNonRoot == 0) expl.push_back(c.name);
    } else if (!podOK) {
      impl.push_back(c.name);
    }
  });
  if (!expl.empty()) setters.push_back(std::string(pluralize("container", "containers", expl.size())) + " " + join_quote(expl));
  if (!setters.empty()) return CR{false, "runAsNonRoot != true", join(setters, " and ") + " must not set securityContext.runAsNonRoot=false"};
  if (!impl.empty())
    return CR{false, "runAsNonRoot != true",
              std::string("pod or ") + pluralize("container", "containers", impl.size()) + " " + join_quote(impl) +
                  " must set securityContext.runAsNonRoot=true"};
  return allowed();
}

CR runAsUser_1_23(const Pod& p) {
  std::vector<std::string> setters, expl;
  if (p.sc.set && p.sc.hasRunAsUser && p.sc.runAsUser == 0) setters.push_back("pod");
  visit_containers(p, [&](const Container& c) {
    if (c.sc.set && c.sc.hasRunAsUser && c.sc.runAsUser == 0) expl.push_back(c.name);
  });
  if (!expl.empty()) setters.push_back(std::string(pluralize("container", "containers", expl.size())) + " " + join_quote(expl));
  if (!setters.empty()) return CR{false, "runAsUser=0", join(setters, " and ") + " must not set runAsUser=0"};
  return allowed();
}

CR seLinuxOptions_1_0(const Pod& p) {
  static const std::set<std::string> okt = {"", "container_t", "container_init_t", "container_kvm_t"};
  std::vector<std::string> setters, badc;
  std::set<std::string> badTypes;
  bool setUser = false, setRole = false;
  auto valid = [&](const SELinux& o) {
    bool v = true;
    if (!okt.count(o.type)) { v = false; badTypes.insert(o.type); }
    if (!o.user.empty()) { v = false; setUser = true; }
    if (!o.role.empty()) { v = false; setRole = true; }
    return v;
  };
  if (p.sc.set && p.sc.selinux.set && !valid(p.sc.selinux)) setters.push_back("pod");
  visit_containers(p, [&](const Container& c) {
    if (c.sc.set && c.sc.selinux.set && !valid(c.sc.selinux)) badc.push_back(c.name);
  });
  if (!badc.empty()) setters.push_back(std::string(pluralize("container", "containers", badc.size())) + " " + join_quote(badc));
  if (!setters.empty()) {
    std::vector<std::string> data;
    if (!badTypes.empty()) data.push_back(std::string(pluralize("type", "types", badTypes.size())) + " " + join_quote(sorted(badTypes)));
    if (setUser) data.push_back("user may not be set");
    if (setRole) data.push_back("role may not be set");
    return CR{false, "seLinuxOptions", join(setters, " and ") + " set forbidden securityContext.seLinuxOptions: " + join(data, "; ")};
  }
  return allowed();
}

bool valid_seccomp(const std::string& t) { return t == "Localhost" || t == "RuntimeDefault"; }

CR seccompProfileBaseline_1_0(const Pod& p) {
  std::set<std::string> forb;
  const std::string podKey = "seccomp.security.alpha.kubernetes.io/pod";
  auto it = p.annotations.find(podKey);
  if (it != p.annotations.end() && it->second == "unconfined") forb.insert(podKey + "=" + gou::go_quote(it->second));
  visit_containers(p, [&](const Container& c) {
    std::string k = "container.seccomp.security.alpha.kubernetes.io/" + c.name;
    auto jt = p.annotations.find(k);
    if (jt != p.annotations.end() && jt->second == "unconfined") forb.insert(k + "=" + gou::go_quote(jt->second));
  });
  if (!forb.empty())
    return CR{false, "seccompProfile",
              std::string("forbidden ") + pluralize("annotation", "annotations", forb.size()) + " " + join(sorted(forb), ", ")};
  return allowed();
}

CR seccompProfileBaseline_1_19(const Pod& p) {
  std::vector<std::string> setters, expl;
  std::set<std::string> vals;
  if (p.sc.set && p.sc.seccomp.set && p.sc.seccomp.type == "Unconfined") { setters.push_back("pod"); vals.insert(p.sc.seccomp.type); }
  visit_containers(p, [&](const Container& c) {
    if (c.sc.set && c.sc.seccomp.set && c.sc.seccomp.type == "Unconfined") { expl.push_back(c.name); vals.insert(c.sc.seccomp.type); }
  });
  if (!expl.empty()) setters.push_back(std::string(pluralize("container", "containers", expl.size())) + " " + join_quote(expl));
  if (!setters.empty())
    return CR{false, "seccompProfile",
              join(setters, " and ") + " must not set securityContext.seccompProfile.type to " + join_quote(sorted(vals))};
  return allowed();
}

CR seccompProfileRestricted_1_19(const Pod& p) {
  std::vector<std::string> setters, expl, impl;
  std::set<std::string> vals;
  bool podSet = false;
  if (p.sc.set && p.sc.seccomp.set) {
    if (!valid_seccomp(p.sc.seccomp.type)) { setters.push_back("pod"); vals.insert(p.sc.seccomp.type); }
    else podSet = true;
  }
  visit_containers(p, [&](const Container& c) {
    if (c.sc.set && c.sc.seccomp.set) {
      if (!valid_seccomp(c.sc.seccomp.type)) { expl.push_back(c.name); vals.insert(c.sc.seccomp.type); }
    } else if (!podSet) {
      impl.push_back(c.name);
    }
  });
  if (!expl.empty()) setters.push_back(std::string(pluralize("container", "containers", expl.size())) + " " + join_quote(expl));
  if (!setters.empty())
    return CR{false, "seccompProfile",
              join(setters, " and ") + " must not set securityContext.seccompProfile.type to " + join_quote(sorted(vals))};
  if (!impl.empty())
    return CR{false, "seccompProfile",
              std::string("pod or ") + pluralize("container", "containers", impl.size()) + " " + join_quote(impl) +
                  " must set securityContext.seccompProfile.type to \"RuntimeDefault\" or \"Localhost\""};
  return allowed();
}
CR seccompProfileRestricted_1_25(const Pod& p) { return windows(p) ? allowed() : seccompProfileRestricted_1_19(p); }

CR sysctls_1_0(const Pod& p) {
  static const std::set<std::string> ok = {"kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range", "net.ipv4.tcp_syncookies",
                                           "net.ipv4.ping_group_range", "net.ipv4.ip_unprivileged_port_start"};
  std::vector<std::string> bad;
  if (p.sc.set) for (auto& s : p.sc.sysctls) if (!ok.count(s)) bad.push_back(s);
  if (!bad.empty()) return CR{false, "forbidden sysctls", join(bad, ", ")};
  return allowed();
}

CR windowsHostProcess_1_0(const Pod& p) {
  std::vector<std::string> bad, setters;
  visit_containers(p, [&](const Container& c) { if (c.sc.set && c.sc.win.set && c.sc.win.hostProcess == 1) bad.push_back(c.name); });
  if (p.sc.set && p.sc.win.set && p.sc.win.hostProcess == 1) setters.push_back("pod");
  if (!bad.empty()) setters.push_back(std::string(pluralize("container", "containers", bad.size())) + " " + join_quote(bad));
  if (!setters.empty()) return CR{false, "hostProcess", join(setters, " and ") + " must not set securityContext.windowsOptions.hostProcess=true"};
  return allowed();
}

struct Check {
  const char* id;
  bool restricted;
  std::vector<CR (*)(const Pod&)> versions;
};

// policy.DefaultChecks(): registration order = init order of check_*.go files (sorted file names)
const std::vector<Check>& default_checks() {
  static const std::vector<Check> c = {
      {"allowPrivilegeEscalation", true, {allowPrivilegeEscalation_1_8, allowPrivilegeEscalation_1_25}},
      {"appArmorProfile", false, {appArmorProfile_1_0}},
      {"capabilities_baseline", false, {capabilitiesBaseline_1_0}},
      {"capabilities_restricted", true, {capabilitiesRestricted_1_22, capabilitiesRestricted_1_25}},
      {"hostNamespaces", false, {hostNamespaces_1_0}},
      {"hostPathVolumes", false, {hostPathVolumes_1_0}},
      {"hostPorts", false, {hostPorts_1_0}},
      {"privileged", false, {privileged_1_0}},
      {"procMount", false, {procMount_1_0}},
      {"restrictedVolumes", true, {restrictedVolumes_1_0}},
      {"runAsNonRoot", true, {runAsNonRoot_1_0}},
      {"runAsUser", true, {runAsUser_1_23}},
      {"seLinuxOptions", false, {seLinuxOptions_1_0}},
      {"seccompProfile_baseline", false, {seccompProfileBaseline_1_0, seccompProfileBaseline_1_19}},
      {"seccompProfile_restricted", true, {seccompProfileRestricted_1_19, seccompProfileRestricted_1_25}},
      {"sysctls", false, {sysctls_1_0}},
      {"windowsHostProcess", false, {windowsHostProcess_1_0}},
  };
  return c;
}

// pkg/pss/utils/mapping.go:45-111
const std::map<std::string, std::vector<std::string>>& controls_to_ids() {
  static const std::map<std::string, std::vector<std::string>> m = {
      {"Capabilities", {"capabilities_baseline", "capabilities_restricted"}},
      {"Seccomp", {"seccompProfile_baseline", "seccompProfile_restricted"}},
      {"Privileged Containers", {"privileged"}},
      {"Host Ports", {"hostPorts"}},
      {"/proc Mount Type", {"procMount"}},
      {"AppArmor", {"appArmorProfile"}},
      {"SELinux", {"seLinuxOptions"}},
      {"Host Namespaces", {"hostNamespaces"}},
      {"HostPath Volumes", {"hostPathVolumes"}},
      {"Sysctls", {"sysctls"}},
      {"HostProcess", {"windowsHostProcess"}},
      {"Privilege Escalation", {"allowPrivilegeEscalation"}},
      {"Running as Non-root", {"runAsNonRoot"}},
      {"Running as Non-root user", {"runAsUser"}},
      {"Volume Types", {"restrictedVolumes"}},
  };
  return m;
}

std::vector<PSSResult> evaluate_pss(const std::string& level, const Pod& pod) {  // evaluate.go:16-37
  std::vector<PSSResult> out;
  for (auto& c : default_checks()) {
    if (level == "baseline" && c.restricted) continue;
    for (auto f : c.versions) {
      CR r = f(pod);
      if (!r.allowed) out.push_back(PSSResult{c.id, r});
    }
  }
  return out;
}

}  // namespace

bool pss_version_ok(const std::string& v) {
  if (v.empty() || v == "latest") return true;
  // api.ParseVersion: ^v1\.(0|[1-9][0-9]*)$
  if (v.size() < 4 || v.compare(0, 3, "v1.") != 0) return false;
  std::string m = v.substr(3);
  if (m.empty()) return false;
  if (m.size() > 1 && m[0] == '0') return false;
  for (char c : m) if (c < '0' || c > '9') return false;
  return m.size() < 10;
}

PSSEval pss_evaluate(const VP& podSecurity, const VP& meta, const VP& spec, const VP& outerMeta) {  // evaluate.go:83-108
  PSSEval ev;
  std::string level = oj::get_str(podSecurity, "level");
  std::string version = oj::get_str(podSecurity, "version");
  if (!pss_version_ok(version)) {
    ev.error = "failed to parse pod security api version: invalid version " + version;
    return ev;
  }
  Pod pod;
  try {
    if (outerMeta && outerMeta != meta) dec_pod(outerMeta, nullptr);
    pod = dec_pod(meta, spec);
  } catch (DecodeError& e) {
    ev.decode_error = e.msg;
    return ev;
  }
  std::vector<PSSResult> res = evaluate_pss(level, pod);
  VP excl = podSecurity ? podSecurity->get("exclude") : nullptr;
  if (excl && excl->t == T::Arr) {
    for (auto& ex : excl->a) {
      std::string control = oj::get_str(ex, "controlName");
      VP images = ex ? ex->get("images") : nullptr;
      std::vector<std::string> pats;
      if (images && images->t == T::Arr) for (auto& i : images->a) pats.push_back(i && i->t == T::Str ? i->s : "");
      Pod sub;
      if (pats.empty()) {  // GetPodWithMatchingContainers: pod-level only
        sub = pod;
        Container fake;
        fake.name = "fake";
        sub.containers = {fake};
        sub.init.clear();
        sub.ephemeral.clear();
      } else {
        sub.name = pod.name;
        sub.ns = pod.ns;
        auto pick = [&](const std::vector<Container>& in, std::vector<Container>& out) {
          for (auto& c : in)
            for (auto& pt : pats)
              if (gou::wildcard_match(pt, c.image)) { out.push_back(c); break; }
        };
        pick(pod.containers, sub.containers);
        pick(pod.init, sub.init);
        pick(pod.ephemeral, sub.ephemeral);
      }
      std::vector<PSSResult> exr = evaluate_pss(level, sub);
      // exemptKyvernoExclusion: map keyed by ID (dedup, last wins; Go map order => ND order)
      std::map<std::string, PSSResult> m;
      for (auto& r : res) m[r.id] = r;
      auto it = controls_to_ids().find(control);
      for (auto& e : exr)
        if (it != controls_to_ids().end())
          for (auto& id : it->second)
            if (e.id == id) m.erase(id);
      res.clear();
      for (auto& kv : m) res.push_back(kv.second);
      ev.order_nondeterministic = true;
    }
  }
  ev.ok = true;
  ev.allowed = res.empty();
  ev.checks = res;
  return ev;
}

std::string format_checks_print(const std::vector<PSSResult>& checks) {  // evaluate.go:160-166
  std::string s;
  for (auto& c : checks)
    s += "({Allowed:" + std::string(c.r.allowed ? "true" : "false") + " ForbiddenReason:" + c.r.reason +
         " ForbiddenDetail:" + c.r.detail + "})\n";
  return s;
}

}  // namespace orc
