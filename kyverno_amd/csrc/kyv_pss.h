// PodSecurity rules on the node table (__host__ __device__).
//
// Restates pkg/pss/evaluate.go (EvaluatePod :83, evaluatePSS :16, exemptKyvernoExclusion :39,
// GetPodWithMatchingContainers :112) and the DefaultChecks() of k8s.io/pod-security-admission v0.26.1
// (module not vendored in the reference; restated from its published algorithm and pinned by
// pkg/pss/evaluate_test.go).  Every check runs ALL of its versions (evaluate.go:24), so the result is a
// bitmask over (check, version) slots in DefaultChecks() registration order.  The typed decode of
// validation.go:481-532 is modelled for the fields the checks read: a JSON type mismatch there is an error.
#pragma once
#include "kyv_cond.h"
#include "kyv_eval.h"
#include "kyv_walk.h"

namespace kyv {

enum PssSlot : uint32_t {
  PS_APE_1_8 = 0, PS_APE_1_25, PS_APPARMOR, PS_CAPS_BASE, PS_CAPS_R_1_22, PS_CAPS_R_1_25, PS_HOSTNS, PS_HOSTPATH,
  PS_HOSTPORTS, PS_PRIVILEGED, PS_PROCMOUNT, PS_RVOLUMES, PS_RUNASNONROOT, PS_RUNASUSER, PS_SELINUX, PS_SECCOMP_B_1_0,
  PS_SECCOMP_B_1_19, PS_SECCOMP_R_1_19, PS_SECCOMP_R_1_25, PS_SYSCTLS, PS_WINHOSTPROCESS, PS_NSLOTS
};
constexpr uint32_t PSS_RESTRICTED_SLOTS = (1u << PS_APE_1_8) | (1u << PS_APE_1_25) | (1u << PS_CAPS_R_1_22) |
                                          (1u << PS_CAPS_R_1_25) | (1u << PS_RVOLUMES) | (1u << PS_RUNASNONROOT) |
                                          (1u << PS_RUNASUSER) | (1u << PS_SECCOMP_R_1_19) | (1u << PS_SECCOMP_R_1_25);

KYV_HD uint32_t get(NodeTab R, uint32_t m, uint32_t key) {
  if (m == NONE || node_type(R[m]) != N_MAP) return NONE;
  return map_find(R, m, key);  // (a linear 16-wide probe of small maps measured 1.5x slower on C2)
}
KYV_HD bool nil(NodeTab R, uint32_t n) { return n == NONE || node_type(R[n]) == N_NULL; }

struct Dec {        // typed-decode validator
  NodeTab R;
  bool bad;
  KYV_HD bool obj(uint32_t n) { if (nil(R, n)) return false; if (node_type(R[n]) != N_MAP) { bad = true; return false; } return true; }
  KYV_HD bool arr(uint32_t n) { if (nil(R, n)) return false; if (node_type(R[n]) != N_ARR) { bad = true; return false; } return true; }
  KYV_HD uint32_t str(uint32_t n) { if (nil(R, n)) return SID_EMPTY; if (node_type(R[n]) != N_STR) { bad = true; return SID_EMPTY; } return R[n].a; }
  KYV_HD int pbool(uint32_t n) {  // -1 nil
    if (nil(R, n)) return -1;
    uint32_t t = node_type(R[n]);
    if (t == N_TRUE) return 1;
    if (t == N_FALSE) return 0;
    bad = true;
    return -1;
  }
  KYV_HD bool i64(uint32_t n, int64_t lo, int64_t hi, int64_t* out) {
    if (nil(R, n)) return false;
    if (node_type(R[n]) != N_INT) { bad = true; return false; }
    int64_t x = (int64_t)(((uint64_t)R[n].b << 32) | R[n].a);
    if (x < lo || x > hi) { bad = true; return false; }
    *out = x;
    return true;
  }
};

struct SecCtx {
  bool set;
  int privileged, ape, runAsNonRoot, hostProcess;
  bool hasRunAsUser;
  int64_t runAsUser;
  bool selSet;
  uint32_t selUser, selRole, selType;
  bool secSet;
  uint32_t secType;
  uint32_t caps;       // capabilities map node or NONE
  bool procSet;
  uint32_t proc;
};

// `full` = false: the typed decode was already verified (RF_PSS_DONE), so fields read only for that validation
// (levels, localhost profiles, gMSA, runAsGroup, readOnlyRootFilesystem, capability strings) are skipped
KYV_HD void dec_selinux(Dec& d, uint32_t n, bool& set, uint32_t& user, uint32_t& role, uint32_t& type, bool full = true) {
  set = d.obj(n);
  user = role = type = SID_EMPTY;
  if (!set) return;
  user = d.str(get(d.R, n, KSID(USER)));
  role = d.str(get(d.R, n, KSID(ROLE)));
  type = d.str(get(d.R, n, KSID(TYPE)));
  if (full) d.str(get(d.R, n, KSID(LEVEL)));
}
KYV_HD void dec_seccomp(Dec& d, uint32_t n, bool& set, uint32_t& type, bool full = true) {
  set = d.obj(n);
  type = SID_EMPTY;
  if (!set) return;
  type = d.str(get(d.R, n, KSID(TYPE)));
  if (full) d.str(get(d.R, n, KSID(LOCALHOSTPROFILE)));
}
KYV_HD int dec_win(Dec& d, uint32_t n, bool full = true) {
  if (!d.obj(n)) return -1;
  int hp = d.pbool(get(d.R, n, KSID(HOSTPROCESS)));
  if (full) {
    d.str(get(d.R, n, KSID(GMSA_NAME)));
    d.str(get(d.R, n, KSID(GMSA)));
    d.str(get(d.R, n, KSID(RUNASUSERNAME)));
  }
  return hp;
}

KYV_HD SecCtx dec_container_sc(Dec& d, uint32_t c, bool full = true) {
  SecCtx s;
  s.set = false; s.privileged = s.ape = s.runAsNonRoot = s.hostProcess = -1; s.hasRunAsUser = false; s.runAsUser = 0;
  s.selSet = false; s.selUser = s.selRole = s.selType = SID_EMPTY; s.secSet = false; s.secType = SID_EMPTY;
  s.caps = NONE; s.procSet = false; s.proc = SID_EMPTY;
  uint32_t sc = get(d.R, c, KSID(SECCTX));
  if (!d.obj(sc)) return s;
  s.set = true;
  NodeTab R = d.R;
  s.privileged = d.pbool(get(R, sc, KSID(PRIVILEGED)));
  s.ape = d.pbool(get(R, sc, KSID(APE)));
  s.runAsNonRoot = d.pbool(get(R, sc, KSID(RUNASNONROOT)));
  if (full) d.pbool(get(R, sc, KSID(READONLYROOTFS)));
  s.hasRunAsUser = d.i64(get(R, sc, KSID(RUNASUSER)), INT64_MIN, INT64_MAX, &s.runAsUser);
  if (full) {
    int64_t g;
    d.i64(get(R, sc, KSID(RUNASGROUP)), INT64_MIN, INT64_MAX, &g);
  }
  dec_selinux(d, get(R, sc, KSID(SELINUX)), s.selSet, s.selUser, s.selRole, s.selType, full);
  dec_seccomp(d, get(R, sc, KSID(SECCOMP)), s.secSet, s.secType, full);
  s.hostProcess = dec_win(d, get(R, sc, KSID(WINOPTS)), full);
  uint32_t caps = get(R, sc, KSID(CAPS));
  if (d.obj(caps)) {
    s.caps = caps;
    if (full) {
      const uint32_t ckeys[2] = {KSID(ADD), KSID(DROP)};
      for (uint32_t key : ckeys) {
        uint32_t l = get(R, caps, key);
        if (d.arr(l)) for (uint32_t i = 0; i < R[l].b; i++) d.str(R[l].a + i);
      }
    }
  }
  uint32_t pm = get(R, sc, KSID(PROCMOUNT));
  if (!nil(R, pm)) { s.procSet = true; s.proc = d.str(pm); }
  return s;
}

// whole-pod typed decode check (fields the checks read, as oracle/opss.cpp dec_pod)
KYV_HD bool decode_ok_meta(Dec& d, uint32_t meta) {
  if (!d.obj(meta)) return !d.bad;
  NodeTab R = d.R;
  d.str(get(R, meta, KSID(NAME)));
  d.str(get(R, meta, KSID(NAMESPACE_KEY)));
  uint32_t ann = get(R, meta, KSID(ANNOTATIONS));
  if (d.obj(ann)) for (uint32_t i = 0; i < R[ann].b; i++) d.str(R[ann].a + i);
  uint32_t lab = get(R, meta, KSID(LABELS));
  if (d.obj(lab)) for (uint32_t i = 0; i < R[lab].b; i++) d.str(R[lab].a + i);
  return !d.bad;
}

KYV_HD void decode_container(Dec& d, uint32_t c) {
  if (!d.obj(c)) return;
  NodeTab R = d.R;
  d.str(get(R, c, KSID(NAME)));
  d.str(get(R, c, KSID(IMAGE)));
  uint32_t ports = get(R, c, KSID(PORTS));
  if (d.arr(ports))
    for (uint32_t i = 0; i < R[ports].b; i++) {
      uint32_t p = R[ports].a + i;
      if (!d.obj(p)) continue;
      int64_t x;
      d.i64(get(R, p, KSID(HOSTPORT)), INT32_MIN, INT32_MAX, &x);
      d.i64(get(R, p, KSID(CONTAINERPORT)), INT32_MIN, INT32_MAX, &x);
      d.str(get(R, p, KSID(NAME)));
      d.str(get(R, p, KSID(PROTOCOL)));
      d.str(get(R, p, KSID(HOSTIP)));
    }
  // the commonly set Container fields beyond what the checks read: []EnvVar{name, value, valueFrom}, command /
  // args []string, workingDir / imagePullPolicy string
  uint32_t env = get(R, c, KSID(ENV));
  if (d.arr(env))
    for (uint32_t i = 0; i < R[env].b; i++) {
      uint32_t e = R[env].a + i;
      if (!d.obj(e)) continue;
      d.str(get(R, e, KSID(NAME)));
      d.str(get(R, e, KSID(VALUE)));
      d.obj(get(R, e, KSID(VALUEFROM)));
    }
  const uint32_t skeys[2] = {KSID(COMMAND), KSID(ARGS)};
  for (uint32_t key : skeys) {
    uint32_t l = get(R, c, key);
    if (d.arr(l)) for (uint32_t i = 0; i < R[l].b; i++) d.str(R[l].a + i);
  }
  d.str(get(R, c, KSID(WORKINGDIR)));
  d.str(get(R, c, KSID(IMAGEPULLPOLICY)));
  dec_container_sc(d, c);
}

KYV_HD bool decode_ok_spec(Dec& d, uint32_t spec) {
  if (!d.obj(spec)) return !d.bad;
  NodeTab R = d.R;
  d.pbool(get(R, spec, KSID(HOSTNETWORK)));
  d.pbool(get(R, spec, KSID(HOSTPID)));
  d.pbool(get(R, spec, KSID(HOSTIPC)));
  uint32_t sc = get(R, spec, KSID(SECCTX));
  if (d.obj(sc)) {
    d.pbool(get(R, sc, KSID(RUNASNONROOT)));
    int64_t x;
    d.i64(get(R, sc, KSID(RUNASUSER)), INT64_MIN, INT64_MAX, &x);
    d.i64(get(R, sc, KSID(RUNASGROUP)), INT64_MIN, INT64_MAX, &x);
    d.i64(get(R, sc, KSID(FSGROUP)), INT64_MIN, INT64_MAX, &x);
    uint32_t sg = get(R, sc, KSID(SUPPGROUPS));
    if (d.arr(sg)) for (uint32_t i = 0; i < R[sg].b; i++) d.i64(R[sg].a + i, INT64_MIN, INT64_MAX, &x);
    bool set; uint32_t a, b, c;
    dec_selinux(d, get(R, sc, KSID(SELINUX)), set, a, b, c);
    dec_seccomp(d, get(R, sc, KSID(SECCOMP)), set, a);
    dec_win(d, get(R, sc, KSID(WINOPTS)));
    uint32_t sy = get(R, sc, KSID(SYSCTLS));
    if (d.arr(sy))
      for (uint32_t i = 0; i < R[sy].b; i++) {
        uint32_t e = R[sy].a + i;
        if (!d.obj(e)) continue;
        d.str(get(R, e, KSID(NAME)));
        d.str(get(R, e, KSID(VALUE)));
      }
  }
  const uint32_t lkeys[3] = {KSID(CONTAINERS), KSID(INITCONTAINERS), KSID(EPHEMERALCONTAINERS)};
  for (uint32_t key : lkeys) {
    uint32_t l = get(R, spec, key);
    if (d.arr(l)) for (uint32_t i = 0; i < R[l].b; i++) decode_container(d, R[l].a + i);
  }
  uint32_t vols = get(R, spec, KSID(VOLUMES));
  if (d.arr(vols))
    for (uint32_t i = 0; i < R[vols].b; i++) {
      uint32_t vn = R[vols].a + i;
      if (!d.obj(vn)) continue;
      d.str(get(R, vn, KSID(NAME)));
      for (uint32_t s = 0; s < V_COUNT; s++) d.obj(get(R, vn, SID_FIRST_FREE + K_COUNT + s));
    }
  uint32_t os = get(R, spec, KSID(OS));
  if (d.obj(os)) d.str(get(R, os, KSID(NAME)));
  // commonly set PodSpec fields beyond what the checks read: nodeSelector map[string]string, serviceAccountName /
  // restartPolicy string, terminationGracePeriodSeconds / activeDeadlineSeconds *int64
  uint32_t ns = get(R, spec, KSID(NODESELECTOR));
  if (d.obj(ns)) for (uint32_t i = 0; i < R[ns].b; i++) d.str(R[ns].a + i);
  d.str(get(R, spec, KSID(SERVICEACCOUNTNAME)));
  d.str(get(R, spec, KSID(RESTARTPOLICY)));
  int64_t t;
  d.i64(get(R, spec, KSID(TGPS)), INT64_MIN, INT64_MAX, &t);
  d.i64(get(R, spec, KSID(ADS)), INT64_MIN, INT64_MAX, &t);
  return !d.bad;
}

// container source of a (sub-)pod: the real lists (optionally filtered by exclusion images) or the
// single fake container of GetPodWithMatchingContainers (evaluate.go:112-146)
struct PodView {
  uint32_t meta;       // NONE for the image-exclusion sub-pod (ObjectMeta{Name, Namespace} only)
  uint32_t spec;       // NONE: pod-level spec fields are empty
  uint32_t lists[3];   // init, containers, ephemeral (visitContainers order)
  bool fake;
  uint32_t img, nimg;  // image globs (pool)
  bool decoded;        // the typed decode was verified by the flattener: the checks skip decode-only fields
};

KYV_HD bool container_included(const View& v, NodeTab R, const PodView& pv, uint32_t c) {
  if (pv.nimg == 0) return true;
  uint32_t image = nil(R, get(R, c, KSID(IMAGE))) ? SID_EMPTY : R[get(R, c, KSID(IMAGE))].a;
  for (uint32_t i = 0; i < pv.nimg; i++) if (glob_sid(v, v.pool[pv.img + i], image)) return true;
  return false;
}

KYV_HD bool str_in(uint32_t s, const uint32_t* set, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) if (set[i] == s) return true;
  return false;
}

KYV_HD bool has_prefix(const View& v, uint32_t s, uint32_t prefix) {
  uint32_t ln = v.str_len[prefix];
  return v.str_len[s] >= ln && bytes_eq(sbytes(v, s), sbytes(v, prefix), ln);
}
// has_prefix for the checks' three fixed prefixes, from the per-string flags (derive_strings)
KYV_HD bool has_pfx(const View& v, uint32_t s, uint32_t flag) { return (v.str_flags[s] & flag) != 0; }

// evaluatePSS (evaluate.go:16-37): failing (check, version) slots
KYV_FN_PSS uint32_t pss_checks(const View& v, NodeTab R, const PodView& pv) {
  Dec d{R, false};
  uint32_t fails = 0;
  uint32_t spec = pv.spec;
  uint32_t psc = get(R, spec, KSID(SECCTX));
  bool pscSet = !nil(R, psc) && node_type(R[psc]) == N_MAP;
  bool windows = false;
  {
    uint32_t os = get(R, spec, KSID(OS));
    uint32_t nm = get(R, os, KSID(NAME));
    windows = !nil(R, nm) && node_type(R[nm]) == N_STR && R[nm].a == KSID(WINDOWS);
  }
  // pod-level security context
  int podNonRoot = pscSet ? d.pbool(get(R, psc, KSID(RUNASNONROOT))) : -1;
  int64_t podUser = 0;
  bool podHasUser = pscSet && d.i64(get(R, psc, KSID(RUNASUSER)), INT64_MIN, INT64_MAX, &podUser);
  const bool full = !pv.decoded;
  bool podSelSet = false; uint32_t pu = SID_EMPTY, pr = SID_EMPTY, pt = SID_EMPTY;
  if (pscSet) dec_selinux(d, get(R, psc, KSID(SELINUX)), podSelSet, pu, pr, pt, full);
  bool podSecSet = false; uint32_t podSecType = SID_EMPTY;
  if (pscSet) dec_seccomp(d, get(R, psc, KSID(SECCOMP)), podSecSet, podSecType, full);
  int podHostProcess = pscSet ? dec_win(d, get(R, psc, KSID(WINOPTS)), full) : -1;

  const uint32_t capsOK[13] = {KSID(CAP_AUDIT_WRITE), KSID(CAP_CHOWN), KSID(CAP_DAC_OVERRIDE), KSID(CAP_FOWNER),
                               KSID(CAP_FSETID), KSID(CAP_KILL), KSID(CAP_MKNOD), KSID(NET_BIND_SERVICE),
                               KSID(CAP_SETFCAP), KSID(CAP_SETGID), KSID(CAP_SETPCAP), KSID(CAP_SETUID),
                               KSID(CAP_SYS_CHROOT)};
  const uint32_t selOK[4] = {SID_EMPTY, KSID(CONTAINER_T), KSID(CONTAINER_INIT_T), KSID(CONTAINER_KVM_T)};
  auto selValid = [&](uint32_t u, uint32_t r, uint32_t t) { return str_in(t, selOK, 4) && u == SID_EMPTY && r == SID_EMPTY; };
  auto secValid = [&](uint32_t t) { return t == KSID(LOCALHOST) || t == KSID(RUNTIMEDEFAULT); };

  // Every flag set inside the container / capability / port / annotation / volume loops is a bit of one integer word
  // (`bad`, `all`, `hn`, `okv`), never a loop-carried bool: divergent loop-carried bools in these nested loops were
  // lowered as lane masks and merged wrongly at divergent loop exits (profiles/r5_pss_miscompile/README.md; the
  // column form pss_checks_cols follows the same rule)
  enum : uint32_t {
    B_APE = 1u << 0, B_CAPS_BASE = 1u << 1, B_CAPS_R = 1u << 2, B_PORTS = 1u << 3, B_PRIV = 1u << 4, B_PROC = 1u << 5,
    B_NONROOT_X = 1u << 6, B_NONROOT_I = 1u << 7, B_USER = 1u << 8, B_SEL = 1u << 9, B_SEC_BASE = 1u << 10,
    B_SEC_RX = 1u << 11, B_SEC_RI = 1u << 12, B_HP = 1u << 13, B_SEC_ANN = 1u << 14
  };
  uint32_t bad = 0;
  bool podNonRootTrue = podNonRoot == 1;
  bool podSecValid = podSecSet && secValid(podSecType);
  uint32_t ann = pv.meta == NONE ? NONE : get(R, pv.meta, KSID(ANNOTATIONS));
  bool annMap = !nil(R, ann) && node_type(R[ann]) == N_MAP;

  auto visit = [&](uint32_t c, bool fake) {
    SecCtx s;
    uint32_t cname = SID_EMPTY;
    if (fake) {
      s.set = false; s.privileged = s.ape = s.runAsNonRoot = s.hostProcess = -1; s.hasRunAsUser = false;
      s.selSet = false; s.secSet = false; s.caps = NONE; s.procSet = false;
      cname = KSID(FAKE);
    } else {
      s = dec_container_sc(d, c, full);
      uint32_t nm = get(R, c, KSID(NAME));
      cname = nil(R, nm) ? SID_EMPTY : R[nm].a;
    }
    if (!s.set || s.ape != 0) bad |= B_APE;
    if (s.set && s.caps != NONE) {
      uint32_t add = get(R, s.caps, KSID(ADD));
      if (!nil(R, add))
        for (uint32_t i = 0; i < R[add].b; i++) {
          uint32_t cap = R[R[add].a + i].a;
          if (node_type(R[R[add].a + i]) != N_STR) cap = SID_EMPTY;
          if (!str_in(cap, capsOK, 13)) bad |= B_CAPS_BASE;
          if (cap != KSID(NET_BIND_SERVICE)) bad |= B_CAPS_R;
        }
      uint32_t all = 0;
      uint32_t drop = get(R, s.caps, KSID(DROP));
      if (!nil(R, drop))
        for (uint32_t i = 0; i < R[drop].b; i++) {
          const Node& e = R[R[drop].a + i];
          if (node_type(e) == N_STR && e.a == KSID(ALL)) all = 1u;
        }
      if (!all) bad |= B_CAPS_R;
    } else {
      bad |= B_CAPS_R;
    }
    if (!fake) {
      uint32_t ports = get(R, c, KSID(PORTS));
      if (!nil(R, ports))
        for (uint32_t i = 0; i < R[ports].b; i++) {
          uint32_t hp = get(R, R[ports].a + i, KSID(HOSTPORT));
          if (!nil(R, hp) && node_type(R[hp]) == N_INT && (R[hp].a | R[hp].b) != 0) bad |= B_PORTS;
        }
    }
    if (s.set && s.privileged == 1) bad |= B_PRIV;
    if (s.set && s.procSet && s.proc != KSID(DEFAULT)) bad |= B_PROC;
    if (s.set && s.runAsNonRoot != -1) { if (s.runAsNonRoot == 0) bad |= B_NONROOT_X; }
    else if (!podNonRootTrue) bad |= B_NONROOT_I;
    if (s.set && s.hasRunAsUser && s.runAsUser == 0) bad |= B_USER;
    if (s.set && s.selSet && !selValid(s.selUser, s.selRole, s.selType)) bad |= B_SEL;
    if (s.set && s.secSet) {
      if (s.secType == KSID(UNCONFINED)) bad |= B_SEC_BASE;
      if (!secValid(s.secType)) bad |= B_SEC_RX;
    } else if (!podSecValid) {
      bad |= B_SEC_RI;
    }
    if (s.set && s.hostProcess == 1) bad |= B_HP;
    // container seccomp annotation: container.seccomp.security.alpha.kubernetes.io/<name> == "unconfined"
    if (annMap) {
      uint32_t pl = v.str_len[KSID(SECCOMP_CONTAINER_PREFIX)], nl = v.str_len[cname];
      for (uint32_t i = 0; i < R[ann].b; i++) {
        const Node& e = R[R[ann].a + i];
        uint32_t k = node_key(e);
        if (has_pfx(v, k, SF_PFX_SECCOMP_C) && v.str_len[k] == pl + nl &&
            bytes_eq(sbytes(v, k) + pl, sbytes(v, cname), nl) && node_type(e) == N_STR && e.a == KSID(UNCONFINED_LC))
          bad |= B_SEC_ANN;
      }
    }
  };
  if (pv.fake) {
    visit(NONE, true);
  } else {
    for (int l = 0; l < 3; l++) {
      uint32_t list = pv.lists[l];
      if (nil(R, list) || node_type(R[list]) != N_ARR) continue;
      for (uint32_t i = 0; i < R[list].b; i++) {
        uint32_t c = R[list].a + i;
        if (!container_included(v, R, pv, c)) continue;
        visit(c, false);
      }
    }
  }
  if (bad & B_APE) fails |= 1u << PS_APE_1_8;
  if ((bad & B_APE) && !windows) fails |= 1u << PS_APE_1_25;
  // appArmorProfile: annotations with the apparmor prefix whose value is neither runtime/default nor localhost/*
  if (annMap)
    for (uint32_t i = 0; i < R[ann].b; i++) {
      const Node& e = R[R[ann].a + i];
      uint32_t val = node_type(e) == N_STR ? e.a : SID_EMPTY;
      if (has_pfx(v, node_key(e), SF_PFX_APPARMOR) && val != KSID(RUNTIME_DEFAULT_PROFILE) &&
          !has_pfx(v, val, SF_PFX_LOCALHOST))
        fails |= 1u << PS_APPARMOR;
      if (node_key(e) == KSID(SECCOMP_POD_ANN) && val == KSID(UNCONFINED_LC)) bad |= B_SEC_ANN;
    }
  if (bad & B_CAPS_BASE) fails |= 1u << PS_CAPS_BASE;
  if (bad & B_CAPS_R) fails |= 1u << PS_CAPS_R_1_22;
  if ((bad & B_CAPS_R) && !windows) fails |= 1u << PS_CAPS_R_1_25;
  {
    uint32_t hn = 0;
    const uint32_t hkeys[3] = {KSID(HOSTNETWORK), KSID(HOSTPID), KSID(HOSTIPC)};
    for (uint32_t key : hkeys) {
      uint32_t n = get(R, spec, key);
      if (!nil(R, n) && node_type(R[n]) == N_TRUE) hn = 1u;
    }
    if (hn) fails |= 1u << PS_HOSTNS;
  }
  uint32_t vols = get(R, spec, KSID(VOLUMES));
  if (!nil(R, vols) && node_type(R[vols]) == N_ARR)
    for (uint32_t i = 0; i < R[vols].b; i++) {
      // one pass over the volume's entries (keys are unique): a non-null hostPath entry, and whether some allowed
      // source (the first V_ALLOWED volume-source sids) is set
      uint32_t vn = R[vols].a + i;
      uint32_t okv = 0;
      if (node_type(R[vn]) == N_MAP)
        for (uint32_t q = 0; q < R[vn].b; q++) {
          const Node& e = R[R[vn].a + q];
          if (node_type(e) == N_NULL) continue;
          const uint32_t k = node_key(e);
          if (k == VSID(hostPath)) fails |= 1u << PS_HOSTPATH;
          if (k >= SID_FIRST_FREE + K_COUNT && k < SID_FIRST_FREE + K_COUNT + V_ALLOWED) okv = 1u;
        }
      if (!okv) fails |= 1u << PS_RVOLUMES;
    }
  if (bad & B_PORTS) fails |= 1u << PS_HOSTPORTS;
  if (bad & B_PRIV) fails |= 1u << PS_PRIVILEGED;
  if (bad & B_PROC) fails |= 1u << PS_PROCMOUNT;
  if (podNonRoot == 0 || (bad & (B_NONROOT_X | B_NONROOT_I))) fails |= 1u << PS_RUNASNONROOT;
  if ((podHasUser && podUser == 0) || (bad & B_USER)) fails |= 1u << PS_RUNASUSER;
  if ((podSelSet && !selValid(pu, pr, pt)) || (bad & B_SEL)) fails |= 1u << PS_SELINUX;
  if (bad & B_SEC_ANN) fails |= 1u << PS_SECCOMP_B_1_0;
  if ((podSecSet && podSecType == KSID(UNCONFINED)) || (bad & B_SEC_BASE)) fails |= 1u << PS_SECCOMP_B_1_19;
  const bool secR = (podSecSet && !secValid(podSecType)) || (bad & (B_SEC_RX | B_SEC_RI));
  if (secR) fails |= 1u << PS_SECCOMP_R_1_19;
  if (secR && !windows) fails |= 1u << PS_SECCOMP_R_1_25;
  if (pscSet) {
    uint32_t sy = get(R, psc, KSID(SYSCTLS));
    const uint32_t ok5[5] = {KSID(SYSCTL_SHM), KSID(SYSCTL_PORTRANGE), KSID(SYSCTL_SYNCOOKIES), KSID(SYSCTL_PINGRANGE),
                             KSID(SYSCTL_UNPRIV)};
    if (!nil(R, sy) && node_type(R[sy]) == N_ARR)
      for (uint32_t i = 0; i < R[sy].b; i++) {
        uint32_t nm = get(R, R[sy].a + i, KSID(NAME));
        uint32_t s = nil(R, nm) ? SID_EMPTY : R[nm].a;
        if (!str_in(s, ok5, 5)) fails |= 1u << PS_SYSCTLS;
      }
  }
  if (podHostProcess == 1 || (bad & B_HP)) fails |= 1u << PS_WINHOSTPROCESS;
  return fails;
}

// pss_checks of the resource's own pod (no exclusion sub-pod) after the typed decode was verified, with every field
// read through its path column (compiler.cpp TrieBuilder::pss_rule; table T of the pod position): the loads of one
// scope are independent (one round for the pod level, one per container) instead of chains of map searches. Same
// semantics as pss_checks(decoded); pinned against it and the oracle by the PodSecurity parity tests.
struct PCol {  // a decoded column entry
  uint32_t i, t, a;  // node index (NONE: absent), node type, the node's `a`
};
KYV_HD PCol pcol(const View& v, uint32_t col, uint32_t row) {
  PCol c{NONE, 0u, 0u};
  if (col == NONE || row == NONE) return c;
  KYV_ACCT_ADD(0, 8);
  const uint64_t x = v.colv[(size_t)v.col_off[col] + row];
  const uint32_t lo = (uint32_t)x;
  if (lo == NONE) return c;
  c.i = lo & COL_INDEX_MASK;
  c.t = lo >> COL_TYPE_SHIFT;
  c.a = (uint32_t)(x >> 32);
  return c;
}
KYV_HD bool pnil(const PCol& c) { return c.i == NONE || c.t == N_NULL; }
KYV_HD int pbool(const PCol& c) { return c.i == NONE ? -1 : c.t == N_TRUE ? 1 : c.t == N_FALSE ? 0 : -1; }
KYV_HD uint32_t pstr(const PCol& c) { return (c.i != NONE && c.t == N_STR) ? c.a : SID_EMPTY; }
KYV_HD bool pobj(const PCol& c) { return c.i != NONE && c.t == N_MAP; }
// an int64 field: present (decoded: an integer) and its value is zero
KYV_HD bool pzero(NodeTab R, const PCol& c) { return c.i != NONE && c.t == N_INT && c.a == 0 && R[c.i].b == 0; }

// the per-container part of the checks (one container: element row `er` of list table L), as fact bits the pod-level
// part combines; F_NRUNSET / F_SECUNSET become failures only when the pod-level field does not supply the value
enum PssFact : uint32_t {
  F_APE = 1u << 0, F_CAPSB = 1u << 1, F_CAPSR = 1u << 2, F_PORTS = 1u << 3, F_PRIV = 1u << 4, F_PROC = 1u << 5,
  F_NREXP = 1u << 6, F_NRUNSET = 1u << 7, F_USER = 1u << 8, F_SEL = 1u << 9, F_SECB = 1u << 10, F_SECREXP = 1u << 11,
  F_SECUNSET = 1u << 12, F_HP = 1u << 13,
};
// a column entry read through the column's absolute colv offset (NONE: no column)
KYV_HD PCol pcol_at(const View& v, uint32_t off, uint32_t row) {
  PCol c{NONE, 0u, 0u};
  if (off == NONE || row == NONE) return c;
  KYV_ACCT_ADD(0, 8);
  const uint64_t x = v.colv[(size_t)off + row];
  const uint32_t lo = (uint32_t)x;
  if (lo == NONE) return c;
  c.i = lo & COL_INDEX_MASK;
  c.t = lo >> COL_TYPE_SHIFT;
  c.a = (uint32_t)(x >> 32);
  return c;
}
// The checks of one container (element row `er`); co(F) is the colv offset of the container list's field F (PCL_*),
// NONE when the table has no such column. pss_container_facts reads the offsets through the list's table words
// (L[F] -> col_off); pss_kernel (round 6), when the wave's pods share their table, passes offsets it read with scalar
// loads, so each field is one vector load instead of a chain of three.
template <class ColOff>
KYV_HD __attribute__((always_inline)) uint32_t pss_container_facts_g(const View& v, NodeTab R, ColOff co, uint32_t er) {
  auto capOK = [](uint32_t c) {
    return (c >= KSID(CAP_AUDIT_WRITE) && c <= KSID(CAP_SYS_CHROOT)) || c == KSID(NET_BIND_SERVICE);
  };
  auto selValid = [&](uint32_t u, uint32_t r, uint32_t t) {
    return (t == SID_EMPTY || (t >= KSID(CONTAINER_T) && t <= KSID(CONTAINER_KVM_T))) && u == SID_EMPTY && r == SID_EMPTY;
  };
  auto secValid = [&](uint32_t t) { return t == KSID(LOCALHOST) || t == KSID(RUNTIMEDEFAULT); };
  uint32_t f = 0;
  // every field of the container: independent loads
  const PCol sc = pcol_at(v, co(PCL_SC), er);
  const PCol priv = pcol_at(v, co(PCL_PRIV), er), ape = pcol_at(v, co(PCL_APE), er), nr = pcol_at(v, co(PCL_NONROOT), er);
  const PCol us = pcol_at(v, co(PCL_USER), er), sel = pcol_at(v, co(PCL_SEL), er), sec = pcol_at(v, co(PCL_SEC), er);
  const PCol win = pcol_at(v, co(PCL_WIN), er), caps = pcol_at(v, co(PCL_CAPS), er), pm = pcol_at(v, co(PCL_PROC), er);
  const uint32_t oadd = co(PCL_ADD_LEN), odrop = co(PCL_DROP_LEN), oport = co(PCL_PORTS_LEN);
  const uint64_t addl = oadd == NONE ? ~0ull : v.colv[(size_t)oadd + er];
  const uint64_t dropl = odrop == NONE ? ~0ull : v.colv[(size_t)odrop + er];
  const uint64_t portl = oport == NONE ? ~0ull : v.colv[(size_t)oport + er];
  KYV_ACCT_ADD(0, 8 * ((oadd != NONE) + (odrop != NONE) + (oport != NONE)));
  const bool set = pobj(sc);
  const int privileged = set ? pbool(priv) : -1, apev = set ? pbool(ape) : -1, nonRoot = set ? pbool(nr) : -1;
  if (!set || apev != 0) f |= F_APE;
  if (set && pobj(caps)) {
    if ((uint32_t)addl != NONE) {
      const uint32_t oself = co(PCL_ADD_SELF);
      for (uint32_t j = 0; j < (uint32_t)addl; j++) {
        const PCol e = pcol_at(v, oself, (uint32_t)(addl >> 32) + j);
        const uint32_t cap = e.t == N_STR ? e.a : SID_EMPTY;
        if (!capOK(cap)) f |= F_CAPSB;
        if (cap != KSID(NET_BIND_SERVICE)) f |= F_CAPSR;
      }
    }
    uint32_t all = 0;  // (loop-carried flags are integer words throughout: see eval_pss)
    if ((uint32_t)dropl != NONE) {
      const uint32_t oself = co(PCL_DROP_SELF);
      for (uint32_t j = 0; j < (uint32_t)dropl; j++) {
        const PCol e = pcol_at(v, oself, (uint32_t)(dropl >> 32) + j);
        if (e.t == N_STR && e.a == KSID(ALL)) all = 1;
      }
    }
    if (!all) f |= F_CAPSR;
  } else {
    f |= F_CAPSR;
  }
  if ((uint32_t)portl != NONE) {
    const uint32_t ohp = co(PCL_PORT_HOSTPORT);
    for (uint32_t j = 0; j < (uint32_t)portl; j++) {
      const PCol hp = pcol_at(v, ohp, (uint32_t)(portl >> 32) + j);
      if (hp.i != NONE && hp.t == N_INT && (hp.a != 0 || R[hp.i].b != 0)) f |= F_PORTS;
    }
  }
  if (set && privileged == 1) f |= F_PRIV;
  if (set && !pnil(pm) && pstr(pm) != KSID(DEFAULT)) f |= F_PROC;
  if (set && nonRoot != -1) { if (nonRoot == 0) f |= F_NREXP; }
  else f |= F_NRUNSET;
  if (set && us.i != NONE && us.t == N_INT && pzero(R, us)) f |= F_USER;
  if (set && pobj(sel) && !selValid(pstr(pcol_at(v, co(PCL_SEL_USER), er)), pstr(pcol_at(v, co(PCL_SEL_ROLE), er)),
                                    pstr(pcol_at(v, co(PCL_SEL_TYPE), er))))
    f |= F_SEL;
  if (set && pobj(sec)) {
    const uint32_t st = pstr(pcol_at(v, co(PCL_SEC_TYPE), er));
    if (st == KSID(UNCONFINED)) f |= F_SECB;
    if (!secValid(st)) f |= F_SECREXP;
  } else {
    f |= F_SECUNSET;
  }
  if (set && pobj(win) && pbool(pcol_at(v, co(PCL_WIN_HP), er)) == 1) f |= F_HP;
  return f;
}
KYV_HD __attribute__((always_inline)) uint32_t pss_container_facts(const View& v, NodeTab R, const uint32_t* L, uint32_t er) {
  return pss_container_facts_g(v, R, [&](uint32_t F) -> uint32_t { return L[F] == NONE ? NONE : v.col_off[L[F]]; }, er);
}

// cf_given: the OR of every container's facts (pss_kernel computes them with one container per lane across the
// wave); else the containers are visited here, one after the other
// po(X): the colv offset of pod field X of table T (NONE: no column) -- pss_checks_cols reads it through the table
// word and col_off; pss_kernel (round 6) passes offsets read with scalar loads when the wave's pods share one table
template <class PodOff>
KYV_HD __attribute__((always_inline)) uint32_t pss_checks_cols_g(const View& v, NodeTab R, uint32_t row, const uint32_t* T,
                                                                PodOff po, uint32_t cf = 0, bool cf_given = false) {
  uint32_t fails = 0;

  const PCol psc = pcol_at(v, po(PC_PSC), row);
  const bool pscSet = pobj(psc);
  const PCol osn = pcol_at(v, po(PC_OS_NAME), row);
  const bool windows = osn.i != NONE && osn.t == N_STR && osn.a == KSID(WINDOWS);
  // pod-level security context (the columns of a non-map securityContext have no entries)
  const PCol pnr = pcol_at(v, po(PC_PSC_NONROOT), row), pus = pcol_at(v, po(PC_PSC_USER), row);
  const PCol psel = pcol_at(v, po(PC_PSC_SEL), row), psec = pcol_at(v, po(PC_PSC_SEC), row), pwin = pcol_at(v, po(PC_PSC_WIN), row);
  const int podNonRoot = pscSet ? pbool(pnr) : -1;
  const bool podHasUser = pscSet && pus.i != NONE && pus.t == N_INT;
  const bool podUserZero = podHasUser && pzero(R, pus);
  const bool podSelSet = pscSet && pobj(psel);
  uint32_t pu = SID_EMPTY, pr = SID_EMPTY, pt = SID_EMPTY;
  if (podSelSet) {
    pu = pstr(pcol_at(v, po(PC_PSC_SEL_USER), row));
    pr = pstr(pcol_at(v, po(PC_PSC_SEL_ROLE), row));
    pt = pstr(pcol_at(v, po(PC_PSC_SEL_TYPE), row));
  }
  const bool podSecSet = pscSet && pobj(psec);
  const uint32_t podSecType = podSecSet ? pstr(pcol_at(v, po(PC_PSC_SEC_TYPE), row)) : SID_EMPTY;
  const int podHostProcess = pscSet && pobj(pwin) ? pbool(pcol_at(v, po(PC_PSC_WIN_HP), row)) : -1;

  // the allowed sets as sid ranges of the seeded well-known strings (no local arrays: they would live in scratch)
  auto capOK = [](uint32_t c) {
    return (c >= KSID(CAP_AUDIT_WRITE) && c <= KSID(CAP_SYS_CHROOT)) || c == KSID(NET_BIND_SERVICE);
  };
  auto selValid = [&](uint32_t u, uint32_t r, uint32_t t) {
    return (t == SID_EMPTY || (t >= KSID(CONTAINER_T) && t <= KSID(CONTAINER_KVM_T))) && u == SID_EMPTY && r == SID_EMPTY;
  };
  auto secValid = [&](uint32_t t) { return t == KSID(LOCALHOST) || t == KSID(RUNTIMEDEFAULT); };

  bool apeBad = false, capsBaseBad = false, capsRBad = false, portsBad = false, privBad = false, procBad = false;
  bool nonRootExplicitBad = false, nonRootImplicitBad = false, userBad = false, selBad = false;
  bool secBaseBad = false, secRExplicitBad = false, secRImplicitBad = false, hpBad = false;
  uint32_t secAnnBad = 0;  // set inside loops: an integer word, not a bool (see eval_pss)
  const bool podNonRootTrue = podNonRoot == 1;
  const bool podSecValid = podSecSet && secValid(podSecType);
  const PCol annc = pcol_at(v, po(PC_ANN), row);
  const uint32_t ann = annc.i;
  const bool annMap = pobj(annc);
  // (round 6) the host-namespace fields, the volumes list and its first two volume nodes are loaded here, beside the
  // annotations map, so the volume chain's first steps overlap the annotation pass instead of following it
  const PCol hnet = pcol_at(v, po(PC_HOSTNET), row), hpid = pcol_at(v, po(PC_HOSTPID), row);
  const PCol hipc = pcol_at(v, po(PC_HOSTIPC), row);
  const PCol vols = pcol_at(v, po(PC_VOLUMES), row);
  const Node vlist = vols.i != NONE && vols.t == N_ARR ? R[vols.i] : Node{N_NULL, 0, 0, 0};
  const uint32_t nvol = node_type(vlist) == N_ARR ? vlist.b : 0u, vol0 = nvol ? vlist.a : 0u;
  Node vpre[2];
#pragma unroll
  for (uint32_t j = 0; j < 2; j++) vpre[j] = j < nvol ? R[vol0 + j] : Node{N_NULL, 0, 0, 0};
  // one pass over the annotations: the appArmor and pod seccomp annotation checks, and whether any key carries the
  // container seccomp prefix (the per-container check below then runs only for such pods)
  uint32_t annSecC = 0;
  // four entries per step: their node rows, then their keys' flag words, as independent loads (a loop of one entry
  // per iteration is a chain of two dependent loads per annotation)
  const uint32_t nann = annMap ? R[ann].b : 0u, ann0 = annMap ? R[ann].a : 0u;
  for (uint32_t q = 0; q < nann; q += 4) {
    Node e[4];
    uint32_t kf[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) e[j] = q + j < nann ? R[ann0 + q + j] : Node{N_NULL, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) kf[j] = q + j < nann ? v.str_flags[node_key(e[j])] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      if (q + j >= nann) break;
      const uint32_t key = node_key(e[j]), val = node_type(e[j]) == N_STR ? e[j].a : SID_EMPTY;
      if ((kf[j] & SF_PFX_APPARMOR) && val != KSID(RUNTIME_DEFAULT_PROFILE) && !has_pfx(v, val, SF_PFX_LOCALHOST))
        fails |= 1u << PS_APPARMOR;
      if (key == KSID(SECCOMP_POD_ANN) && val == KSID(UNCONFINED_LC)) secAnnBad = 1;
      if (kf[j] & SF_PFX_SECCOMP_C) annSecC = 1;
    }
  }

  // the containers: facts (given, or gathered here) and, for pods with container seccomp annotations, the per-name
  // annotation check (container.seccomp.security.alpha.kubernetes.io/<name> == "unconfined")
  for (uint32_t l = 0; l < PSS_NLISTS && (!cf_given || annSecC); l++) {
    const uint32_t* L = T + PC_LISTS + l * PCL_COUNT;
    if (L[PCL_LEN] == NONE) continue;
    KYV_ACCT_ADD(0, 8);
    const uint64_t ln = v.colv[(size_t)v.col_off[L[PCL_LEN]] + row];  // (count, row of element 0)
    if ((uint32_t)ln == NONE) continue;  // absent, null or not an array (length entries: NONE count)
    const uint32_t cnt = (uint32_t)ln, eb = (uint32_t)(ln >> 32);
    for (uint32_t i = 0; i < cnt; i++) {
      const uint32_t er = eb + i;
      if (!cf_given) cf |= pss_container_facts(v, R, L, er);
      if (annSecC) {
        const PCol nm = pcol(v, L[PCL_NAME], er);
        const uint32_t cname = nm.i == NONE || nm.t == N_NULL ? SID_EMPTY : nm.a;
        const uint32_t pl = v.str_len[KSID(SECCOMP_CONTAINER_PREFIX)], nl = v.str_len[cname];
        for (uint32_t q = 0; q < R[ann].b; q++) {
          const Node& e = R[R[ann].a + q];
          const uint32_t k = node_key(e);
          if (has_pfx(v, k, SF_PFX_SECCOMP_C) && v.str_len[k] == pl + nl &&
              bytes_eq(sbytes(v, k) + pl, sbytes(v, cname), nl) && node_type(e) == N_STR && e.a == KSID(UNCONFINED_LC))
            secAnnBad = 1;
        }
      }
    }
  }
  apeBad = cf & F_APE; capsBaseBad = cf & F_CAPSB; capsRBad = cf & F_CAPSR; portsBad = cf & F_PORTS;
  privBad = cf & F_PRIV; procBad = cf & F_PROC; nonRootExplicitBad = cf & F_NREXP;
  nonRootImplicitBad = (cf & F_NRUNSET) && !podNonRootTrue; userBad = cf & F_USER; selBad = cf & F_SEL;
  secBaseBad = cf & F_SECB; secRExplicitBad = cf & F_SECREXP; secRImplicitBad = (cf & F_SECUNSET) && !podSecValid;
  hpBad = cf & F_HP;
  if (apeBad) fails |= 1u << PS_APE_1_8;
  if (apeBad && !windows) fails |= 1u << PS_APE_1_25;
  if (capsBaseBad) fails |= 1u << PS_CAPS_BASE;
  if (capsRBad) fails |= 1u << PS_CAPS_R_1_22;
  if (capsRBad && !windows) fails |= 1u << PS_CAPS_R_1_25;
  if (hnet.t == N_TRUE || hpid.t == N_TRUE || hipc.t == N_TRUE) fails |= 1u << PS_HOSTNS;
  // two volumes per step, and each volume's first four entries (name and source) with them: the loads of one step
  // are independent of each other (the first step's volume nodes were loaded before the annotation pass)
  auto vol_entry = [&](const Node& e, uint32_t* okv) {
    if (node_type(e) == N_NULL) return;
    const uint32_t k = node_key(e);
    if (k == VSID(hostPath)) fails |= 1u << PS_HOSTPATH;
    if (k >= SID_FIRST_FREE + K_COUNT && k < SID_FIRST_FREE + K_COUNT + V_ALLOWED) *okv = 1;
  };
  for (uint32_t i = 0; i < nvol; i += 2) {
    Node vn[2];
#pragma unroll
    for (uint32_t j = 0; j < 2; j++) vn[j] = i == 0 ? vpre[j] : i + j < nvol ? R[vol0 + i + j] : Node{N_NULL, 0, 0, 0};
    Node en[2][4];
#pragma unroll
    for (uint32_t j = 0; j < 2; j++)
#pragma unroll
      for (uint32_t q = 0; q < 4; q++)
        en[j][q] = node_type(vn[j]) == N_MAP && q < vn[j].b ? R[vn[j].a + q] : Node{N_NULL, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < 2; j++) {
      if (i + j >= nvol) break;
      uint32_t okv = 0;
      if (node_type(vn[j]) == N_MAP) {
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) vol_entry(en[j][q], &okv);
        for (uint32_t q = 4; q < vn[j].b; q++) vol_entry(R[vn[j].a + q], &okv);
      }
      if (!okv) fails |= 1u << PS_RVOLUMES;
    }
  }
  if (portsBad) fails |= 1u << PS_HOSTPORTS;
  if (privBad) fails |= 1u << PS_PRIVILEGED;
  if (procBad) fails |= 1u << PS_PROCMOUNT;
  if (podNonRoot == 0 || nonRootExplicitBad || nonRootImplicitBad) fails |= 1u << PS_RUNASNONROOT;
  if (podUserZero || userBad) fails |= 1u << PS_RUNASUSER;
  if ((podSelSet && !selValid(pu, pr, pt)) || selBad) fails |= 1u << PS_SELINUX;
  if (secAnnBad) fails |= 1u << PS_SECCOMP_B_1_0;
  if ((podSecSet && podSecType == KSID(UNCONFINED)) || secBaseBad) fails |= 1u << PS_SECCOMP_B_1_19;
  const bool secR = (podSecSet && !secValid(podSecType)) || secRExplicitBad || secRImplicitBad;
  if (secR) fails |= 1u << PS_SECCOMP_R_1_19;
  if (secR && !windows) fails |= 1u << PS_SECCOMP_R_1_25;
  if (pscSet) {
    const PCol sy = pcol_at(v, po(PC_PSC_SYSCTLS), row);
    if (sy.i != NONE && sy.t == N_ARR)
      for (uint32_t i = 0; i < R[sy.i].b; i++) {
        const uint32_t nm = get(R, R[sy.i].a + i, KSID(NAME));
        const uint32_t sname = nil(R, nm) ? SID_EMPTY : R[nm].a;
        if (!(sname >= KSID(SYSCTL_SHM) && sname <= KSID(SYSCTL_UNPRIV))) fails |= 1u << PS_SYSCTLS;
      }
  }
  if (podHostProcess == 1 || hpBad) fails |= 1u << PS_WINHOSTPROCESS;
  return fails;
}

KYV_HD __attribute__((always_inline)) uint32_t pss_checks_cols(const View& v, NodeTab R, uint32_t row, const uint32_t* T,
                                                              uint32_t cf = 0, bool cf_given = false) {
  return pss_checks_cols_g(v, R, row, T, [&](uint32_t X) -> uint32_t { return T[X] == NONE ? NONE : v.col_off[T[X]]; },
                           cf, cf_given);
}

// check-id groups: slots belonging to one check ID (exemptKyvernoExclusion removes whole IDs)
KYV_HD uint32_t pss_id_slots(uint32_t slot) {
  switch (slot) {
    case PS_APE_1_8: case PS_APE_1_25: return (1u << PS_APE_1_8) | (1u << PS_APE_1_25);
    case PS_CAPS_R_1_22: case PS_CAPS_R_1_25: return (1u << PS_CAPS_R_1_22) | (1u << PS_CAPS_R_1_25);
    case PS_SECCOMP_B_1_0: case PS_SECCOMP_B_1_19: return (1u << PS_SECCOMP_B_1_0) | (1u << PS_SECCOMP_B_1_19);
    case PS_SECCOMP_R_1_19: case PS_SECCOMP_R_1_25: return (1u << PS_SECCOMP_R_1_19) | (1u << PS_SECCOMP_R_1_25);
    default: return 1u << slot;
  }
}

// getSpec (validation.go:481-532) for a PodSecurity rule: the pod (template) of the resource's kind, typed-decoded
// when `decode`. ST_NONE: *meta / *spec are its metadata and spec nodes; ST_ERROR: it does not decode; ST_PANIC: a
// kind without a pod spec (nil dereference, validation.go:542-543)
KYV_HD uint8_t pss_pod(NodeTab R, uint32_t kind, bool decode, uint32_t* meta_out, uint32_t* spec_out) {
  uint32_t root = 0;
  uint32_t meta = NONE, spec = NONE;
  Dec d{R, false};
  uint32_t outerMeta = get(R, root, KSID(METADATA));
  auto step = [&](uint32_t o, uint32_t k) -> uint32_t {
    if (d.bad || nil(R, o)) return NONE;
    if (node_type(R[o]) != N_MAP) { d.bad = true; return NONE; }
    uint32_t x = map_find(R, o, k);
    if (!nil(R, x) && node_type(R[x]) != N_MAP) { d.bad = true; return NONE; }
    return x;
  };
  if (!nil(R, outerMeta) && node_type(R[outerMeta]) != N_MAP) d.bad = true;
  if (kind == KSID(DAEMONSET) || kind == KSID(DEPLOYMENT) || kind == KSID(JOB) || kind == KSID(STATEFULSET) ||
      kind == KSID(REPLICASET) || kind == KSID(RC)) {
    uint32_t tpl = step(step(root, KSID(SPEC)), KSID(TEMPLATE));
    meta = step(tpl, KSID(METADATA));
    spec = step(tpl, KSID(SPEC));
  } else if (kind == KSID(CRONJOB)) {
    uint32_t jt = step(step(root, KSID(SPEC)), KSID(JOBTEMPLATE));
    meta = step(jt, KSID(METADATA));
    spec = step(step(step(jt, KSID(SPEC)), KSID(TEMPLATE)), KSID(SPEC));
  } else if (kind == KSID(POD)) {
    meta = outerMeta;
    spec = step(root, KSID(SPEC));
  } else {
    return ST_PANIC;  // nil pod spec dereference (validation.go:542-543)
  }
  if (d.bad) return ST_ERROR;
  *meta_out = meta;
  *spec_out = spec;
  if (!decode) return ST_NONE;
  if (outerMeta != meta && !nil(R, outerMeta) && !decode_ok_meta(d, outerMeta)) return ST_ERROR;
  if (!decode_ok_meta(d, meta) || !decode_ok_spec(d, spec)) return ST_ERROR;
  return ST_NONE;
}

// the column form's preconditions: ST_NONE with *T = the pod position's column table when the checks run over path
// columns; ST_ERROR / ST_PANIC / ST_FALLBACK when that is the pair's status already; ST_PSS_MAP when the column form
// does not apply (exclusion sub-pods, no columns, typed decode not done)
KYV_HD uint8_t pss_cols_table(const View& v, const PssDesc& pd, const ResHeader& h, const uint32_t** T) {
  *T = nullptr;
  if (pd.flags & PSS_BAD_VERSION) return ST_ERROR;
  if (!(h.flags & RF_PSS_DONE) || pd.cols == NONE || pd.nexcl != 0 || !v.colv || h.nnodes >= (1u << COL_TYPE_SHIFT))
    return ST_PSS_MAP;
  if (h.flags & RF_PSS_DEC_ERR) return ST_ERROR;
  if (h.flags & RF_PSS_FOLD) return KYV_WHY(FBW_COND), ST_FALLBACK;
  const uint32_t pos = h.kind == KSID(POD) ? 0u
                     : (h.kind == KSID(DAEMONSET) || h.kind == KSID(DEPLOYMENT) || h.kind == KSID(JOB) ||
                        h.kind == KSID(STATEFULSET) || h.kind == KSID(REPLICASET) || h.kind == KSID(RC)) ? 1u
                     : h.kind == KSID(CRONJOB) ? 2u : NONE;
  if (pos == NONE) return ST_PANIC;  // no pod spec for this kind (validation.go:542-543)
  const uint32_t* t = v.pool + pd.cols + pos * PC_COUNT;
  if (t[PC_PSC] == NONE) return ST_PSS_MAP;  // the table lacks this position (the rule's kinds)
  *T = t;
  return ST_NONE;
}

// validatePodSecurity (validation.go:535-566) over path columns -> status; *fails_out receives the remaining failing
// slots; ST_NONE with *fails_out = 0 when the column form does not apply (the caller then takes the map walk). row: the
// resource's batch position (its column row), passed explicitly by every caller
KYV_HD __attribute__((always_inline)) uint8_t eval_pss_cols(const View& v, const PssDesc& pd, const ResHeader& h,
                                                            NodeTab R, uint32_t* fails_out, uint32_t row) {
  *fails_out = 0;
  const uint32_t* T;
  const uint8_t pre = pss_cols_table(v, pd, h, &T);
  if (pre == ST_PSS_MAP) return ST_NONE;
  if (pre != ST_NONE) return pre;
  const uint32_t mask = (pd.flags & PSS_BASELINE) ? ~PSS_RESTRICTED_SLOTS : 0xFFFFFFFFu;
  const uint32_t fails = pss_checks_cols(v, R, row, T) & mask;
  *fails_out = fails;
  return fails ? ST_FAIL : ST_PASS;
}

// Loop-carried flags of the PodSecurity checks are integer words, never bools. Rounds 3 / 4 kept the column checks out
// of line in eval_pss because, inlined there (eval_pss is itself a call from match_kernel), the device set the
// capabilities / hostPorts failure bits of pods that have neither. Round 5 found the cause on the MI355X with the
// round-4 source ("PodSecurity miscompile"): the loaded values were right (hashes of every list-length,
// port and capability entry equal on host and device) and no loop ran past its lane's trip count (guards on
// optimiser-opaque copies), but the divergent bools set inside the nested container / capability / port loops came out
// set for lanes that never set them: the lowering of loop-carried divergent i1 values (lane masks merged across nested
// divergent loops) in the inlined, call-containing function. The same source with those flags as uint32_t words is
// correct inlined, so the checks are inlined again, with every loop-carried flag an integer word.
KYV_FN_PSS uint8_t eval_pss(const View& v, const PssDesc& pd, NodeTab R, const ResHeader& h, uint32_t* fails_out,
                            uint32_t row) {
  *fails_out = 0;
  if (pd.flags & PSS_BAD_VERSION) return ST_ERROR;
  // the typed decode was done by the flattener when it could (RF_PSS_DONE); else here
  const bool done = (h.flags & RF_PSS_DONE) != 0;
  {
    const uint8_t c = eval_pss_cols(v, pd, h, R, fails_out, row);  // path-column form when it applies
    if (c != ST_NONE) return c;
  }
  uint32_t meta = NONE, spec = NONE;
  const uint8_t ps = pss_pod(R, h.kind, !done, &meta, &spec);
  if (ps != ST_NONE) return ps;
  if (done && (h.flags & RF_PSS_DEC_ERR)) return ST_ERROR;
  if (done && (h.flags & RF_PSS_FOLD)) return KYV_WHY(FBW_COND), ST_FALLBACK;
  PodView pv;
  pv.meta = meta;
  pv.spec = spec;
  pv.lists[0] = get(R, spec, KSID(INITCONTAINERS));
  pv.lists[1] = get(R, spec, KSID(CONTAINERS));
  pv.lists[2] = get(R, spec, KSID(EPHEMERALCONTAINERS));
  pv.fake = false;
  pv.img = 0;
  pv.nimg = 0;
  pv.decoded = done;  // (a decode error returned above)
  uint32_t mask = (pd.flags & PSS_BASELINE) ? ~PSS_RESTRICTED_SLOTS : 0xFFFFFFFFu;
  uint32_t fails = pss_checks(v, R, pv) & mask;
  for (uint32_t x = 0; x < pd.nexcl; x++) {
    // exclusion record in pool: [control slot mask, nimages, image sids...]
    uint32_t rec = v.pool[pd.excl + x];
    uint32_t ctl = v.pool[rec], nimg = v.pool[rec + 1];
    PodView sub = pv;
    if (nimg == 0) {
      sub.fake = true;
    } else {
      sub.meta = NONE;
      sub.spec = NONE;
      sub.img = rec + 2;
      sub.nimg = nimg;
    }
    uint32_t ex = pss_checks(v, R, sub) & mask;
    for (uint32_t s = 0; s < PS_NSLOTS; s++)
      if ((ctl >> s) & 1u) {
        uint32_t ids = pss_id_slots(s);
        if (ex & ids) fails &= ~ids;
      }
  }
  *fails_out = fails;
  return fails ? ST_FAIL : ST_PASS;
}

}  // namespace kyv

namespace kyv {


// validateForEach (validation.go:319-341) + validateElements (:343-381), nested foreach included: each element of
// the evaluated list (evaluateList, utils.go:343-355: a non-list result is a one-element list; a query error skips the
// entry) gets its own validator (newForEachValidator :242-275, validate :276-317): its preconditions (not met -> the
// element is skipped), then deny conditions (true -> the rule fails), or a pattern / anyPattern (validatePatterns
// :618-702 on the element when it is element-scoped -- a map, unless elementScope says otherwise (addElementToContext
// :383-413) -- else on what the enclosing level validates: the resource at the top, the enclosing scoped element
// inside a nested foreach, since PolicyContext.Copy keeps it), or a nested foreach over the element. A failing
// element fails the rule; an error ends it only on the last element; a skipped element is not applied; no applied
// element at all -> "rule skipped".
// Element values enter patterns through the JSON context (numbers float64): an element variable of a pattern
// (L_DYN) is resolved per element (a key missing on the way is the fork's NotFoundError -> the substitution fails:
// an error for this element).
struct FeCtx {
  uint32_t el;    // enclosing element (node, JMES_KEYBIT key) or NONE at the top
  uint32_t root;  // the node a non-scoped element's pattern validates
};

// the value of element variable `d` (pool: kind, nseg, segs...) for element `el` at list position `idx`; false when a
// key is missing on the way (NotFoundError)
KYV_HD bool fe_dyn_value(const View& v, NodeTab R, const uint32_t* d, uint32_t el, uint32_t idx, Val* out) {
  if (d[0] == 1) {  // elementIndex: a number
    *out = value_of(v, R, NONE);
    out->t = N_FLOAT;
    out->f = (double)idx;
    return true;
  }
  uint32_t cur = el;
  Val key{};
  bool is_key = false;
  for (uint32_t s = 0; s < d[1]; s++) {
    if (cur == NONE || (cur & JMES_KEYBIT) || node_type(R[cur]) != N_MAP) { cur = NONE; break; }  // field of a non-map
    const uint32_t x = map_find(R, cur, d[2 + s]);
    if (x == NONE) return false;
    cur = x;
  }
  if (cur != NONE && (cur & JMES_KEYBIT)) {  // the element is a map key (keys(@) list): a string
    is_key = true;
    key = value_of(v, R, NONE);
    key.t = N_STR;
    key.sid = key.wsid = key.nsid = node_key(R[cur & ~JMES_KEYBIT]);
  }
  *out = is_key ? key : value_of(v, R, cur);
  if (out->t == 0xFF) out->t = N_NULL;  // a null value
  return true;
}

// one entry list at nesting level D (levels beyond FOREACH_MAX_NEST never occur: the compiler keeps them on the CPU
// engine; each level is its own instantiation, so only kernels with nested rules carry the deeper levels)
template <int D>
KYV_HD uint8_t foreach_level(const View& v, NodeTab R, const RuleDesc& rd, uint32_t entries, FeCtx up, uint32_t row) {
  if constexpr (D > (int)FOREACH_MAX_NEST) {
    return KYV_WHY(FBW_COND), ST_FALLBACK;
  } else {
    const uint32_t nent = v.pool[entries];
    uint32_t applied = 0;
    for (uint32_t e = 0; e < nent; e++) {
      const ForeachEntry fe = *(const ForeachEntry*)(v.pool + entries + 1 + e * (sizeof(ForeachEntry) / 4));
      JList L;
      JRes lr;
      lr.lst = false; lr.cur = NONE; lr.lit = NONE; lr.num = NONE;
      uint32_t miss = 0;
      if (fe.list.kind == OK_PATH) {
        uint32_t cur = 0;
        bool nf = false;
        for (uint32_t s = 0; s < fe.list.nseg && cur != NONE; s++) {
          bool missing;
          cur = j_field(R, cur, v.pool[fe.list.a + s], &missing);
          if (missing) nf = true;
        }
        if (nf) continue;  // NotFoundError: "failed to evaluate list" -> next entry
        lr.cur = cur;
      } else {
        const int st = jmes_run(v, R, fe.list, up.el, L, &lr, &miss);
        if (st == JS_NOTFOUND || st == JS_ERR || st == JS_TERR) continue;  // "failed to evaluate list": next entry
        if (st == JS_FB) return KYV_WHY(FBW_COND), ST_FALLBACK;
        if (lr.lit != NONE || lr.num != NONE) return KYV_WHY(FBW_COND), ST_FALLBACK;  // literal / number: not restated
      }
      // elements: the projection list, an array's items, or the single value
      const bool arr = !lr.lst && j_arr(R, lr.cur);
      const uint32_t n = lr.lst ? L.n : arr ? R[lr.cur].b : 1u;
      uint32_t count = 0;
      for (uint32_t j = 0; j < n; j++) {
        const uint32_t el = lr.lst ? L.e[j] : arr ? R[lr.cur].a + j : lr.cur;
        if (el == NONE || (!(el & JMES_KEYBIT) && node_type(R[el]) == N_NULL)) continue;
        const bool is_map = j_map(R, el);
        if (fe.scope == 2 && !is_map) return ST_ERROR | ST_MARK_SCOPE;  // addElementToContext error
        const bool scoped = fe.scope == 0 ? is_map : fe.scope == 2;
        const uint32_t target = scoped ? el : up.root;
        uint32_t ec, es, eg;
        uint8_t r = ST_PASS;  // the element validator's response (ST_NONE: no validator)
        bool err = false;
        if (fe.pre != NONE) {
          const int c = eval_prog(v, R, fe.pre, &ec, &es, &eg, el, row);
          if (c == CR_FB) return KYV_WHY(FBW_COND), ST_FALLBACK;
          if (c == CR_PANIC) return ST_PANIC;
          if (c == CR_FALSE) continue;  // "preconditions not met": skip, not applied
          err = c == CP_ERROR;
        }
        if (err) {
          r = ST_ERROR;
        } else if (fe.kind == FE_DENY) {
          const int c = eval_prog(v, R, fe.deny, &ec, &es, &eg, el, row);
          if (c == CR_FB) return KYV_WHY(FBW_COND), ST_FALLBACK;
          if (c == CR_PANIC) return ST_PANIC;
          r = c == CR_TRUE ? ST_FAIL : c == CP_ERROR ? ST_ERROR : ST_PASS;
        } else if (fe.kind == FE_PATTERN || fe.kind == FE_ANYPATTERN) {
          Val dyn[MAX_DYN];
          bool subst_ok = true;
          if (fe.dyn != NONE) {
            const uint32_t nd = v.pool[fe.dyn];
            uint32_t at = fe.dyn + 1;
            for (uint32_t q = 0; q < nd && q < MAX_DYN && subst_ok; q++) {
              subst_ok = fe_dyn_value(v, R, v.pool + at, el, j, &dyn[q]);
              at += 2 + v.pool[at + 1];
            }
          }
          if (!subst_ok) {
            r = ST_ERROR;  // "variable substitution failed" (validation.go:294-297)
          } else {
            Frame frames[MAX_DEPTH];
            const ResHeader& h = v.hdr[row];
            const bool pat = fe.kind == FE_PATTERN;
            const uint32_t nalts = pat ? 1u : fe.nalts;
            uint32_t nfail = 0, nskip = 0;
            r = ST_NONE;
            for (uint32_t a = 0; a < nalts && r == ST_NONE; a++) {
              PatOut po;
              po.status = ST_NONE;
              eval_pattern(v, pat ? fe.body : v.pool[fe.body + a], R, h, rd, Stack{frames, 1, MAX_DEPTH}, po, target,
                           fe.dyn != NONE ? dyn : nullptr);
              switch (po.status) {
                case ST_PASS: r = ST_PASS; break;
                case ST_SKIP: nskip++; break;
                case ST_FAIL: nfail++; break;
                case ST_ERROR: if (pat) r = ST_ERROR; else nfail++; break;  // anyPattern: a path-less error is a fail
                default: return po.status;  // fallback / panic / nondeterministic
              }
            }
            if (r == ST_NONE) r = nfail ? ST_FAIL : nskip ? ST_SKIP : (pat ? ST_FAIL : ST_PASS);
          }
        } else if (fe.kind == FE_NESTED) {
          const uint8_t x = foreach_level<D + 1>(v, R, rd, fe.body, FeCtx{el, target}, row);
          switch (x & 7) {
            case ST_PASS: case ST_SKIP: case ST_FAIL: case ST_ERROR: r = x & 7; break;
            default: return x;  // fallback / panic / nondeterministic
          }
        } else {
          continue;  // no validator: "skip rule due to empty result"
        }
        if (r == ST_SKIP) continue;
        if (r == ST_PASS) { count++; continue; }
        if (r == ST_FAIL) return ST_FAIL;
        if (j + 1 < n) continue;  // an error ends the rule only on the last element
        return ST_ERROR;
      }
      applied += count;
    }
    return applied ? ST_PASS : ST_SKIP;
  }
}

KYV_HD uint8_t eval_foreach(const View& v, NodeTab R, const RuleDesc& rd, uint32_t row = NONE) {
  return foreach_level<0>(v, R, rd, rd.root, FeCtx{NONE, 0u}, row);
}

// The match part of pair_dispatch (validation.go:134-183, matches with the OldResource retry :600-615): false with
// *st = the pair's final status (not matched, nondeterministic, fallback), true when the rule body runs
KYV_HD bool pair_match(const View& v, uint32_t r, const RuleDesc& rd, uint8_t* st) {
  if (rd.match.mode == MM_NONE) { *st = ST_FALLBACK; return KYV_WHY(FBW_MATCH), false; }  // match program not compiled
  if (!(rd.flags & RD_GATE_EXACT)) KYV_ACCT_ADD(0, 16);  // header words the match program compares (model)
  const ResHeader& h = v.hdr[r];
  NodeTab R{v.nodes + h.root};
  LabelSet nsl{NodeTab{nullptr}, 0, nullptr, 0};
  if (h.nsl != NONE) { nsl.kv = v.nsl_kv + 2 * v.nsl_off[h.nsl]; nsl.n = v.nsl_off[h.nsl + 1] - v.nsl_off[h.nsl]; }
  bool nd = false;
  bool m = true;  // RD_GATE_EXACT: the kind gate already decided the match
  if (!(rd.flags & RD_GATE_EXACT)) {
    m = match_rule(v, rd, ResView{R, &h}, nsl, &nd);
    if (!m && rd.empty_may_match) m = match_rule(v, rd, ResView{R, nullptr}, nsl, &nd);
  }
  if (!m) { *st = ST_NONE; return false; }
  if (nd) { *st = ST_ND; return false; }
  if (rd.exc != NONE) {  // hasPolicyExceptions (validation.go:158-161, :797-848): the first candidate that matches
    const uint32_t* e = v.pool + rd.exc;
    const uint32_t n = e[0];
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t* c = e + 1 + 3 * i;
      if (match_exception(v, c[0], c[1], c[2], ResView{R, &h}, nsl, &nd)) {
        *st = nd ? (uint8_t)ST_ND : (uint8_t)(ST_SKIP | ((i + 1u) << 3));
        return false;
      }
    }
    if (nd) { *st = ST_ND; return false; }
  }
  if (rd.kind == RK_FALLBACK) { *st = ST_FALLBACK; return false; }
  return true;
}

// Match + dispatch of one pair (validation.go:134-183, :276-317). Returns the verdict, or sets *walk for a
// pattern / anyPattern pair whose verdict comes from the pattern walk (pair_walk).
// kJ = false: the light instantiation (no JMESPath operands, no foreach) for rules the host classified as such
template <bool kJ = true>
KYV_HD uint8_t pair_dispatch(const View& v, bool active, uint32_t r, uint32_t k, uint32_t* pss_fails, bool* walk) {
  *pss_fails = 0;
  *walk = false;
  const RuleDesc& rd = v.rules[k];
  uint8_t st = ST_NONE;
  if (!active) return st;
  if (!pair_match(v, r, rd, &st)) return st;
  const ResHeader& h = v.hdr[r];
  NodeTab R{v.nodes + h.root};
  uint32_t ec, es, eg;
  // checkPreconditions (validation.go:281-288), then for a deny rule validateDeny (validation.go:437-464): one
  // program evaluation site for both (pass 0 / 1), inlined
  const uint32_t p0 = rd.pre != NONE ? 0u : 1u, p1 = rd.kind == RK_DENY ? 2u : 1u;
  for (uint32_t pass = p0; pass < p1; pass++) {
    const int c = eval_prog_inl<kJ>(v, R, pass ? rd.root : rd.pre, &ec, &es, &eg, NONE, r);
    if (c == CR_FB) return KYV_WHY(FBW_COND), ST_FALLBACK;
    if (c == CR_PANIC) return ST_PANIC;
    if (pass == 0) {
      if (c == CP_ERROR) return ST_ERROR | ST_MARK_PRE;
      if (c == CR_FALSE) return ST_SKIP | ST_MARK_PRE;
    } else {
      if (c == CP_ERROR) return ST_ERROR;
      return c == CR_TRUE ? ST_FAIL : ST_PASS;
    }
  }
  switch (rd.kind) {
    case RK_PANIC: return ST_PANIC;
    case RK_ERROR: return ST_ERROR;
    case RK_DENY: return ST_NONE;  // (decided above)
    case RK_PSS: return eval_pss(v, v.pss[rd.root], R, h, pss_fails, r);
    case RK_FOREACH:
      if constexpr (kJ) return eval_foreach(v, R, rd, r);
      else return ST_FALLBACK;
    case RK_PATTERN: case RK_ANYPATTERN:
      if (h.flags & RF_MAGIC) return KYV_WHY(FBW_PHRASE), ST_FALLBACK;
      *walk = true;
      return ST_NONE;
    default: return ST_NONE;
  }
}

// One (resource, rule) pair end to end (host backend)
template <class Sink, class Walker>
KYV_HD uint8_t eval_pair(const View& v, bool active, uint32_t r, uint32_t k, Walker& wk, uint32_t* pss_fails, Sink& sink) {
  bool walk = false;
  uint8_t st = pair_dispatch(v, active, r, k, pss_fails, &walk);
  const RuleDesc& rd = v.rules[k];
  if (rd.kind != RK_PATTERN && rd.kind != RK_ANYPATTERN) return st;
  uint8_t ws = pair_walk(v, rd, walk, r, k, walk ? v.nodes + v.hdr[r].root : nullptr, wk, sink);
  return walk ? ws : st;
}

}  // namespace kyv
