// Device-resident data layout shared by the host compiler/flattener and the HIP kernels.
//
// Resources ("batch"): every resource is a position-independent table of 16-byte nodes in DFS order;
// container children (map entries / array elements) are contiguous, addressed relative to the resource
// root, and map entries are sorted by key id so a key lookup can stop early.  All strings (keys and
// values, plus the decimal / %E / %f renderings of numbers) are interned in one per-batch dictionary
// whose first entries are the ruleset's literals, so equality tests are id compares and only wildcard
// globs touch string bytes.
//
// Rules ("ruleset"): each validate rule is compiled to a match program (filters over resource header
// columns) plus either a pattern program (pnodes/entries/leaves/atoms, traversal order fully resolved at
// compile time, reference validate/utils.go:36-58) or a PodSecurity descriptor.
#pragma once
#ifndef __HIPCC_RTC__
#include <cstdint>
#else
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::size_t size_t;
#ifndef INT64_MAX
#define INT64_MAX 9223372036854775807LL
#define INT64_MIN (-INT64_MAX - 1)
#define INT32_MAX 2147483647
#define INT32_MIN (-INT32_MAX - 1)
#endif
#endif

namespace kyv {

constexpr uint32_t NONE = 0xFFFFFFFFu;

// ---------------------------------------------------------------- resource nodes
enum NodeType : uint32_t { N_NULL = 0, N_FALSE = 1, N_TRUE = 2, N_INT = 3, N_FLOAT = 4, N_STR = 5, N_MAP = 6, N_ARR = 7 };

struct Node {     // 16 bytes
  uint32_t tk;    // type (low 4 bits) | key sid << 4 (map entries) / array index << 4 (array elements)
  uint32_t a;     // MAP/ARR: first child (relative); STR: sid; INT/FLOAT: low 32 bits; BOOL: 0/1
  uint32_t b;     // MAP/ARR: child count; INT/FLOAT: high 32 bits
  uint32_t c;     // INT: sid of decimal form; FLOAT: index into float aux table; ARR: path-column row of
                  // element 0 (NONE when no pattern reads inside this array); STR/MAP: unused
};
static_assert(sizeof(Node) == 16, "node size");

inline constexpr uint32_t node_type(const Node& n) { return n.tk & 0xF; }
inline constexpr uint32_t node_key(const Node& n) { return n.tk >> 4; }

struct FloatAux {   // per float node: string forms interned in the dictionary
  uint32_t sid_E;   // strconv.FormatFloat(v,'E',-1,64)  (compareString, pattern.go:272)
  uint32_t sid_F;   // fmt "%f"                           (convertNumberToString, pattern.go:311)
};

// per-dictionary-string flags
enum StrFlag : uint32_t {
  SF_ASCII = 1u << 0,
  SF_DUR = 1u << 1,        // time.ParseDuration ok
  SF_QTY = 1u << 2,        // resource.ParseQuantity ok and representable as int128 nano units
  SF_QTY_BIG = 1u << 3,    // ParseQuantity ok but beyond int128 nano -> pair falls back
  SF_FLOAT = 1u << 4,      // strconv.ParseFloat ok
  SF_LKEY = 1u << 5,       // valid label key (IsQualifiedName)
  SF_LVAL = 1u << 6,       // valid label value
  SF_MAGIC = 1u << 7,      // contains an anchor-error phrase (error.go:20-26)
  SF_INT = 1u << 8,        // strconv.ParseInt(s, 10, 64) ok (value = str_f64 when not SF_INT_BIG)
  SF_INT_BIG = 1u << 9,    // ... but |value| > 2^53 (not exact in str_f64) -> condition pairs fall back
  SF_SEMVERISH = 1u << 10, // could parse as blang/semver (digit first, two dots) -> numeric conditions fall back
  SF_GLOBBY = 1u << 11,    // as a wildcard pattern it needs the rune matcher: holds '*' or '?', or is not ASCII
                           // (else wildcard.Match(p, s) is p == s, i.e. an id compare)
  // PodSecurity annotation prefixes (the checks' strings.HasPrefix, decided once per string)
  SF_PFX_APPARMOR = 1u << 12,   // "container.apparmor.security.beta.kubernetes.io/"
  SF_PFX_LOCALHOST = 1u << 13,  // "localhost/"
  SF_PFX_SECCOMP_C = 1u << 14,  // "container.seccomp.security.alpha.kubernetes.io/"
  // as a pattern string s, validateStringPatterns(v, s) (pattern.go:152-301) is "v is the string s, or a bool whose
  // strconv.FormatBool is s": ASCII, no '|' '&' '*' '?', no leading / trailing blank, no operator prefix
  // ('<' '>' '!'), no digit / sign / '.' first (range, duration and quantity forms). A foreach pattern leaf
  // substituted from an element variable (L_DYN) is decided on the device only for such strings
  SF_PLAIN = 1u << 15,
};
// bits 16..23 of a ruleset wildcard pattern's str_flags: its glob-mask index + 1 (0: none). The device holds one
// bit per (dictionary string, masked pattern): wildcard.Match(pattern, string), evaluated once per batch
// (kyv_engine.hip gmask_kernel), so a glob test is one load instead of a byte loop over the heap
constexpr uint32_t SF_GIDX_SHIFT = 16;
constexpr uint32_t MAX_GMASK = 128;  // masked patterns per ruleset (4 words per string); the rest match bytes

// fixed dictionary ids (seeded first in every batch)
enum FixedSid : uint32_t { SID_EMPTY = 0, SID_ZERO = 1, SID_TRUE = 2, SID_FALSE = 3, SID_STAR = 4, SID_FIRST_FREE = 5 };

// resource flags
enum ResFlag : uint32_t {
  RF_MAGIC = 1u << 0,       // some string/key contains an anchor-error phrase, or a map/array exceeds 65535
                            // entries -> pattern pairs fall back
  RF_ANCHORISH = 1u << 1,   // some key under metadata parses as an anchor -> metadata expansion falls back
  RF_EMPTY = 1u << 2,
  RF_TOO_DEEP = 1u << 3,
  RF_ROOT_MAP = 1u << 4,    // the resource document is a JSON object (walks skip the root row's type check load)
  // metadata of the resource root as wildcards.go ExpandInMetadata type-asserts it (for expansion sites without
  // wildcard keys the compiled walk decides from these flags instead of re-reading the maps):
  RF_META_NONE = 1u << 5,   // metadata absent or null
  RF_META_NOTMAP = 1u << 6, // metadata present, not an object
  RF_LAB_BAD = 1u << 7,     // metadata.labels present, not null, and not an object of strings
  RF_ANN_BAD = 1u << 8,     // metadata.annotations likewise
  // typed decode of the pod (template) a PodSecurity rule reads (validation.go:481-532), done once per resource by
  // the flattener when the ruleset has PodSecurity rules (RF_PSS_DONE): RF_PSS_DEC_ERR = it does not decode
  RF_PSS_DONE = 1u << 9,
  RF_PSS_DEC_ERR = 1u << 10,
  // it decodes, but some key of the object matched its Go field only case-insensitively (encoding/json's fold match):
  // the checks read exact keys, so the resource's PodSecurity pairs go back to the caller (ST_FALLBACK)
  RF_PSS_FOLD = 1u << 19,
};
// the same four metadata flags (NONE, NOTMAP, LAB_BAD, ANN_BAD as consecutive bits) for the pod templates of the
// autogen'd rules: spec.template.metadata at RF_TMETA1_SHIFT, spec.jobTemplate.spec.template.metadata at
// RF_TMETA2_SHIFT (the resource root's are bits 5..8)
constexpr uint32_t RF_META_SHIFT = 5, RF_TMETA1_SHIFT = 11, RF_TMETA2_SHIFT = 15;

struct ResHeader {          // 64 bytes, one per resource (unstructured accessors, host-computed)
  uint32_t root;            // node offset of the resource root in the batch node array
  uint32_t nnodes;
  uint32_t kind;            // GetKind()
  uint32_t gvk_kind;        // GroupVersionKind().Kind ("" when apiVersion does not parse)
  uint32_t group, version;  // parsed apiVersion
  uint32_t gv;              // GroupVersion().String()
  uint32_t name, gen_name, ns;
  uint32_t labels;          // relative node of metadata.labels when it is a map of strings, else NONE
  uint32_t ann;             // same for annotations
  uint32_t nsl;             // namespace-label set id, NONE if unknown
  uint32_t flags;
  uint32_t orig;            // index of the resource in the caller's input order
  uint32_t kclass;          // kind class (row of the batch's rule gate table)
};
static_assert(sizeof(ResHeader) == 64, "header size");

// ---------------------------------------------------------------- match programs
enum MatchMode : uint8_t { MM_NONE = 0, MM_PLAIN = 1, MM_ANY = 2, MM_ALL = 3,
                           MM_EXC_ALL = 4 };  // a PolicyException match with neither any nor all: matches everything

enum FilterFlag : uint16_t {
  FF_ZERO_RD = 1 << 0,        // ResourceDescription is the zero value
  FF_USERINFO = 1 << 1,       // roles / clusterRoles / subjects present (never satisfied in background scans)
  FF_KINDS_STAR = 1 << 2,     // kinds contains "*"
  FF_SEL_INVALID = 1 << 3,    // selector statically invalid -> CheckSelector error
  FF_NSSEL_INVALID = 1 << 4,
  FF_HAS_SEL = 1 << 5,
  FF_HAS_NSSEL = 1 << 6,
};

struct KindDesc {         // compiled kinds[] entry (pkg/utils/kube/kind.go GetKindFromGVK)
  uint32_t kind;          // sid of the kind part (exact compare against ResHeader.gvk_kind); NONE for "*"
  uint32_t gv_mode;       // 0 none, 1 exact group/version, 2 prefix (gv contains '*'), 3 invalid gv (never)
  uint32_t g, v;          // mode 1: group/version sids; mode 2: g = prefix string sid
};

struct Filter {
  uint16_t flags;
  uint16_t nkinds;
  uint32_t kinds;          // first KindDesc
  uint32_t name;           // glob sid or NONE
  uint32_t names, nnames;  // sids in u32 pool
  uint32_t nss, nnss;
  uint32_t ann, nann;      // pairs (key glob sid, value glob sid) in u32 pool
  uint32_t sel, nsel;      // selector descriptors
};

enum ReqOp : uint32_t { RQ_EQ = 0, RQ_IN = 1, RQ_NOTIN = 2, RQ_EXISTS = 3, RQ_NOTEXISTS = 4, RQ_WILD = 5 };
struct SelReq {            // one requirement; values in u32 pool
  uint32_t op;
  uint32_t key;            // key sid (RQ_WILD: key glob sid)
  uint32_t vals, nvals;    // RQ_WILD: vals = value glob sid
  uint32_t rkey, rval;     // RQ_WILD: replacement ('*','?' -> '0') key/value sids, NONE if statically invalid
};
struct SelDesc {
  uint32_t reqs, nreqs;
  uint32_t invalid;        // statically invalid (-> error)
  uint32_t pad;
};

struct MatchBlock {
  uint8_t mode;
  uint8_t pad[3];
  uint32_t filters, nfilters;
};

// ---------------------------------------------------------------- pattern programs
enum PKind : uint8_t { P_MAP = 0, P_ARR_MAPS = 1, P_ARR_SCALAR = 2, P_ARR_POS = 3, P_ARR_EMPTY = 4, P_LEAF = 5 };
enum PFlag : uint8_t { PF_META = 1, PF_NEEDROW = 2 };  // PF_NEEDROW: map has an entry without a path column

struct PNode {          // 16 bytes
  uint8_t kind;
  uint8_t flags;
  uint8_t level;        // ARR_MAPS: dynamic index slot
  uint8_t meta;         // PF_META: metadata-expansion site id
  uint32_t first;       // MAP: first entry; ARR_MAPS/ARR_SCALAR: child pnode; ARR_POS: first of n consecutive pnode ids in pool; LEAF: leaf id
  uint32_t n;           // MAP: entries; ARR_POS: pattern elements
  uint32_t tmpl;        // path template of this node
};

enum Handler : uint8_t { H_DEFAULT = 0, H_STAR = 1, H_EQUALITY = 2, H_CONDITION = 3, H_GLOBAL = 4, H_NEGATION = 5,
                         H_EXISTENCE = 6, H_EXIST_BADPAT = 7 };
enum EntryFlag : uint8_t { EF_WILD = 1 };  // key resolved at run time by metadata expansion (slot in `slot`)

struct PEntry {         // 20 bytes
  uint8_t handler;
  uint8_t flags;
  uint8_t abit;         // anchor-map bit (0xFF none)
  uint8_t slot;         // EF_WILD: expansion slot
  uint32_t key;         // sid looked up in the resource map
  uint32_t child;       // child pnode (EXISTENCE: first of n pattern maps in pool, n in `tmpl_n`)
  uint32_t tmpl;        // currentPath template (path + key + "/")
  uint32_t col;         // path column holding this lookup's result per row of the map's row space, or NONE
};

// Path columns ("columnar JSON-path tables"). Every static key path the ruleset's patterns look up is a
// column: for each row of its row space, an 8-byte entry: low word = the resolved node (type << COL_TYPE_SHIFT |
// node index relative to the resource root) or NONE, high word = the node's `a` (string id, first child, ...).
// Row space 0 is the resource (row = resource position in the batch); every pattern array position ("[*]" in
// the path trie) opens a row space whose rows are the elements of all resource arrays at that path, numbered
// batch-wide, with a "self" column holding each element; an array node's `c` holds the row of its element 0.
constexpr uint32_t COL_TYPE_SHIFT = 28;
constexpr uint32_t COL_INDEX_MASK = (1u << COL_TYPE_SHIFT) - 1;

// L_DYN: a foreach pattern value that is exactly one element variable ({{element...}} / {{elementIndex}}); `exact`
// holds its slot in the entry's dynamic-value list, resolved per element before the walk (vars.go:352-431 substitutes
// a whole-string variable by its typed value)
enum LeafType : uint8_t { L_NIL = 0, L_BOOL = 1, L_FLOAT = 2, L_STR = 3, L_MAP = 4, L_ARR = 5, L_DYN = 6 };
constexpr uint32_t FOREACH_MAX_NEST = 3;  // nested foreach levels below the top the device evaluates (deeper -> CPU)
constexpr uint32_t MAX_DYN = 4;  // element variables per foreach pattern entry (more -> CPU fallback)
struct Leaf {           // 32 bytes
  uint8_t type;
  uint8_t bval;
  uint8_t fint;         // float pattern is integral
  uint8_t pad;
  uint32_t exact;       // L_STR: sid of the whole pattern string
  uint32_t groups, ngroups;  // L_STR: OR-groups (each: atoms start,count in u32 pool pairs)
  double f;
  int64_t fi;           // int64(pattern) (Go conversion)
};

enum AtomOp : uint8_t { A_EQ = 0, A_NE = 1, A_GT = 2, A_LT = 3, A_GE = 4, A_LE = 5, A_RANGE_IN = 6, A_RANGE_OUT = 7, A_FALSE = 8 };
enum GlobKind : uint8_t { G_ANY = 0, G_EMPTY = 1, G_EXACT = 2, G_PREFIX = 3, G_SUFFIX = 4, G_CONTAINS = 5, G_NONEMPTY = 6,
                          G_GENERAL = 7 };
enum AtomFlag : uint8_t { AF_DUR = 1, AF_QTY = 2 };

struct Atom {           // 48 bytes; range atoms reference two simple atoms (a, a+1)
  uint8_t op;
  uint8_t flags;
  uint8_t glob;
  uint8_t gidx;         // glob-mask index + 1 of `pat` (PREFIX/SUFFIX/CONTAINS/GENERAL), 0 none
  uint32_t pat;         // sid of the (trimmed) pattern string for compareString
  uint32_t lit;         // sid of the literal part for PREFIX/SUFFIX/CONTAINS
  uint32_t sub;         // RANGE_*: index of first of two sub-atoms
  int64_t dur;
  int64_t qlo, qhi;     // int128 nano units
};

struct MetaSite {       // metadata-expansion site (wildcards.go:62-83)
  uint32_t has_labels;  // pattern metadata carries a labels / annotations map (type-asserted at run time)
  uint32_t has_ann;
  uint32_t wild_l, nwild_l;  // wildcard entries (u32 pool pairs): key glob sid, unresolved key sid
  uint32_t wild_a, nwild_a;
  uint32_t slot_l, slot_a;   // first slot ids
};

// well-known strings, seeded right after the fixed sids in every dictionary (K_x sid = SID_FIRST_FREE + x)
#define KYV_WELL_KNOWN(X)                                                                                    \
  X(METADATA, "metadata") X(LABELS, "labels") X(ANNOTATIONS, "annotations") X(SPEC, "spec")                 \
  X(TEMPLATE, "template") X(JOBTEMPLATE, "jobTemplate") X(POD, "Pod") X(CRONJOB, "CronJob")                 \
  X(DAEMONSET, "DaemonSet") X(DEPLOYMENT, "Deployment") X(JOB, "Job") X(STATEFULSET, "StatefulSet")          \
  X(REPLICASET, "ReplicaSet") X(RC, "ReplicationController") X(NAMESPACE, "Namespace")                      \
  X(CONTAINERS, "containers") X(INITCONTAINERS, "initContainers") X(EPHEMERALCONTAINERS, "ephemeralContainers") \
  X(NAME, "name") X(IMAGE, "image") X(PORTS, "ports") X(HOSTPORT, "hostPort") X(SECCTX, "securityContext")   \
  X(PRIVILEGED, "privileged") X(APE, "allowPrivilegeEscalation") X(RUNASNONROOT, "runAsNonRoot")            \
  X(RUNASUSER, "runAsUser") X(SELINUX, "seLinuxOptions") X(SECCOMP, "seccompProfile") X(TYPE, "type")       \
  X(USER, "user") X(ROLE, "role") X(CAPS, "capabilities") X(ADD, "add") X(DROP, "drop")                     \
  X(PROCMOUNT, "procMount") X(WINOPTS, "windowsOptions") X(HOSTPROCESS, "hostProcess")                     \
  X(HOSTNETWORK, "hostNetwork") X(HOSTPID, "hostPID") X(HOSTIPC, "hostIPC") X(SYSCTLS, "sysctls")         \
  X(VOLUMES, "volumes") X(OS, "os") X(WINDOWS, "windows") X(ALL, "ALL")             \
  X(NET_BIND_SERVICE, "NET_BIND_SERVICE") X(LOCALHOST, "Localhost") X(RUNTIMEDEFAULT, "RuntimeDefault")     \
  X(UNCONFINED, "Unconfined") X(DEFAULT, "Default") X(RUNTIME_DEFAULT_PROFILE, "runtime/default")           \
  X(UNCONFINED_LC, "unconfined") X(SECCOMP_POD_ANN, "seccomp.security.alpha.kubernetes.io/pod")             \
  X(LEVEL, "level") X(VALUE, "value") X(CONTAINERPORT, "containerPort") X(PROTOCOL, "protocol")             \
  X(HOSTIP, "hostIP") X(RUNASGROUP, "runAsGroup") X(FSGROUP, "fsGroup") X(SUPPGROUPS, "supplementalGroups")  \
  X(READONLYROOTFS, "readOnlyRootFilesystem") X(LOCALHOSTPROFILE, "localhostProfile")                       \
  X(GMSA_NAME, "gmsaCredentialSpecName") X(GMSA, "gmsaCredentialSpec") X(RUNASUSERNAME, "runAsUserName")     \
  X(NAMESPACE_KEY, "namespace") X(APPARMOR_PREFIX, "container.apparmor.security.beta.kubernetes.io/")        \
  X(LOCALHOST_PREFIX, "localhost/") X(SECCOMP_CONTAINER_PREFIX, "container.seccomp.security.alpha.kubernetes.io/") \
  X(CONTAINER_T, "container_t") X(CONTAINER_INIT_T, "container_init_t") X(CONTAINER_KVM_T, "container_kvm_t") \
  X(CAP_AUDIT_WRITE, "AUDIT_WRITE") X(CAP_CHOWN, "CHOWN") X(CAP_DAC_OVERRIDE, "DAC_OVERRIDE")               \
  X(CAP_FOWNER, "FOWNER") X(CAP_FSETID, "FSETID") X(CAP_KILL, "KILL") X(CAP_MKNOD, "MKNOD")                  \
  X(CAP_SETFCAP, "SETFCAP") X(CAP_SETGID, "SETGID") X(CAP_SETPCAP, "SETPCAP") X(CAP_SETUID, "SETUID")        \
  X(CAP_SYS_CHROOT, "SYS_CHROOT") X(SYSCTL_SHM, "kernel.shm_rmid_forced")                                    \
  X(SYSCTL_PORTRANGE, "net.ipv4.ip_local_port_range") X(SYSCTL_SYNCOOKIES, "net.ipv4.tcp_syncookies")        \
  X(SYSCTL_PINGRANGE, "net.ipv4.ping_group_range") X(SYSCTL_UNPRIV, "net.ipv4.ip_unprivileged_port_start")   \
  X(FAKE, "fake") X(NIL_STR, "<nil>")                                                                        \
  X(ENV, "env") X(VALUEFROM, "valueFrom") X(COMMAND, "command") X(ARGS, "args") X(WORKINGDIR, "workingDir")   \
  X(IMAGEPULLPOLICY, "imagePullPolicy") X(NODESELECTOR, "nodeSelector") X(SERVICEACCOUNTNAME, "serviceAccountName") \
  X(RESTARTPOLICY, "restartPolicy") X(TGPS, "terminationGracePeriodSeconds") X(ADS, "activeDeadlineSeconds")

enum WellKnown : uint32_t {
#define KYV_WK_ENUM(id, s) K_##id,
  KYV_WELL_KNOWN(KYV_WK_ENUM)
#undef KYV_WK_ENUM
  K_COUNT
};
#define KSID(id) (SID_FIRST_FREE + K_##id)
// sid ranges the path-column PodSecurity checks test (kyv_pss.h pss_checks_cols)
static_assert(K_CAP_SYS_CHROOT - K_CAP_AUDIT_WRITE == 11 && K_CONTAINER_KVM_T - K_CONTAINER_T == 2 &&
              K_SYSCTL_UNPRIV - K_SYSCTL_SHM == 4, "well-known string ranges");

// typed VolumeSource members: the 8 allowed by restrictedVolumes first, then the reference switch order
// used to name a forbidden source (pod-security-admission policy/check_restrictedVolumes.go)
#define KYV_VOLUME_SOURCES(X)                                                                                \
  X(configMap) X(csi) X(downwardAPI) X(emptyDir) X(ephemeral) X(persistentVolumeClaim) X(projected) X(secret) \
  X(hostPath) X(gcePersistentDisk) X(awsElasticBlockStore) X(gitRepo) X(nfs) X(iscsi) X(glusterfs) X(rbd)     \
  X(flexVolume) X(cinder) X(cephfs) X(flocker) X(fc) X(azureFile) X(vsphereVolume) X(quobyte) X(azureDisk)    \
  X(photonPersistentDisk) X(portworxVolume) X(scaleIO) X(storageos)
enum VolumeSource : uint32_t {
#define KYV_VS_ENUM(id) V_##id,
  KYV_VOLUME_SOURCES(KYV_VS_ENUM)
#undef KYV_VS_ENUM
  V_COUNT
};
constexpr uint32_t V_ALLOWED = 8;
#define VSID(id) (SID_FIRST_FREE + K_COUNT + V_##id)
constexpr uint32_t SID_SEED_END = SID_FIRST_FREE + K_COUNT + V_COUNT;

// ---------------------------------------------------------------- PodSecurity
enum PssFlag : uint32_t { PSS_BASELINE = 1, PSS_BAD_VERSION = 2 };
struct PssDesc {
  uint32_t flags;
  uint32_t excl, nexcl;  // exclusions (u32 pool): control bits, nimages, images...
  uint32_t cols;         // pool offset of the path-column table [PSS_NPOS][PC_COUNT] (NONE: the checks search maps)
};

// Path columns of the fields the PodSecurity checks read (compiler.cpp TrieBuilder::pss), per pod position of getSpec
// (validation.go:481-532): 0 Pod (metadata / spec at the root), 1 pod template (spec.template), 2 CronJob
// (spec.jobTemplate.spec.template). Pod-level fields live in the resource row space; container fields in the row
// space of their list's elements (three lists: initContainers, containers, ephemeralContainers -- visitContainers
// order); array fields carry their length column (count, element-0 row) and their elements' self column.
constexpr uint32_t PSS_NPOS = 3;
enum PssCol : uint32_t {
  PC_ANN = 0, PC_PSC, PC_PSC_NONROOT, PC_PSC_USER, PC_PSC_SEL, PC_PSC_SEL_USER, PC_PSC_SEL_ROLE, PC_PSC_SEL_TYPE,
  PC_PSC_SEC, PC_PSC_SEC_TYPE, PC_PSC_WIN, PC_PSC_WIN_HP, PC_PSC_SYSCTLS, PC_OS_NAME, PC_HOSTNET, PC_HOSTPID,
  PC_HOSTIPC, PC_VOLUMES, PC_LISTS,  // then PSS_NLISTS x PCL_COUNT list columns
};
enum PssListCol : uint32_t {
  PCL_LEN = 0, PCL_SELF, PCL_NAME, PCL_SC, PCL_PRIV, PCL_APE, PCL_NONROOT, PCL_USER, PCL_SEL, PCL_SEL_USER, PCL_SEL_ROLE,
  PCL_SEL_TYPE, PCL_SEC, PCL_SEC_TYPE, PCL_WIN, PCL_WIN_HP, PCL_CAPS, PCL_ADD_LEN, PCL_ADD_SELF, PCL_DROP_LEN,
  PCL_DROP_SELF, PCL_PROC, PCL_PORTS_LEN, PCL_PORT_HOSTPORT, PCL_COUNT
};
constexpr uint32_t PSS_NLISTS = 3;
constexpr uint32_t PC_COUNT = PC_LISTS + PSS_NLISTS * PCL_COUNT;

// ---------------------------------------------------------------- rules
enum RuleKind : uint8_t { RK_NONE = 0, RK_PATTERN = 1, RK_ANYPATTERN = 2, RK_PSS = 3, RK_FALLBACK = 4, RK_PANIC = 5,
                          RK_ERROR = 6, RK_DENY = 7, RK_FOREACH = 8 };

// ---------------------------------------------------------------- conditions (validate.deny, rule preconditions)
// A condition program is the any/all form of pkg/engine/variables/evaluate.go:42-69 (the old list form is an `all`
// block without `any`). Operands are literals (ruleset node table `cnodes`, already put through the
// Condition.GetKey json round trip) or `{{ request.object.<path> }}` references resolved per resource.
enum CondOp : uint8_t { CO_EQ = 0, CO_NE = 1, CO_IN = 2, CO_NOTIN = 3, CO_ANYIN = 4, CO_ALLIN = 5, CO_ANYNOTIN = 6,
                        CO_ALLNOTIN = 7, CO_GT = 8, CO_GE = 9, CO_LT = 10, CO_LE = 11, CO_FALSE = 12,
                        CO_DGT = 13, CO_DGE = 14, CO_DLT = 15, CO_DLE = 16 };  // Duration* (operator/duration.go)
enum OperandKind : uint8_t { OK_NIL = 0, OK_LIT = 1, OK_PATH = 2, OK_JMES = 3 };

// JMESPath-subset operand program (OK_JMES; pool words at CondOperand.a, CondOperand.nseg words): go-jmespath
// sub-expressions, multi-select lists, flatten projections, keys(@) and a trailing `|| <literal>`, linearised at
// compile time. Word 0 is the root; then ops (opcode word + operands). Inside these programs a key missing from a
// map is null (the kyverno/go-jmespath fork's NotFoundError applies to plain field chains only: JR flag JF_PURE).
enum JmesRoot : uint32_t { JR_OBJECT = 0, JR_ELEMENT = 1, JR_OPERATION = 2 };
constexpr uint32_t JF_PURE = 1u << 8;      // root word flag: plain field chain (missing key -> NotFoundError)
enum JmesOp : uint32_t { JO_FIELD = 1,     // + key sid
                         JO_MULTI = 2,     // + n, n key sids   (multi-select list of fields)
                         JO_FLAT = 3,      // flatten projection (nulls dropped)
                         JO_KEYS = 4,      // keys(@) of the current map
                         JO_KEYS_FLAT = 5, // projection keys(@) then flatten
                         JO_OR = 6,        // + cnode literal: `|| <literal>` when the result is false-like
                         JO_LENGTH = 7,    // length(<the ops before>): a number (go-jmespath jpfLength)
                         JO_FILTER = 8,    // + FilterKind, literal, n, n key sids: filter projection `[?<pred>]`
                         JO_UPPER = 9,     // to_upper(<the ops before>): Batch::str_upper of the string (round 6)
                         JO_REGEX = 10 };  // + q: regex_match(<ruleset regex q>, <the ops before>): bit q of Batch::str_rx
// filter predicates the device evaluates per element (the compiler keeps other predicates on the CPU engine):
//   FK_HASKEY  contains(keys(@), '<lit>')  literal = key sid; an element that is not a map: keys() type error
//   FK_EQ/NE   <field chain> == / != <literal>  literal = cnode (string, boolean or null)
enum FilterKind : uint32_t { FK_HASKEY = 0, FK_EQ = 1, FK_NE = 2 };
// words of the op at p (opcode + operands)
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
__host__ __device__
#endif
inline uint32_t jop_width(const uint32_t* p) {
  return p[0] == JO_FIELD || p[0] == JO_OR || p[0] == JO_REGEX ? 2u : p[0] == JO_MULTI ? 2u + p[1] :
         p[0] == JO_FILTER ? 4u + p[3] : 1u;
}
// Programs the light kernels evaluate without the interpreter's list state (kyv_cond.h jmes_chain_cv): a field chain
// of request.object, an optional `|| literal`, and an optional function applied last -- length() (go-jmespath
// jpfLength), to_upper() / regex_match() (kyverno pkg/engine/jmespath/functions.go:681-689, 786-799):
//   [JR_OBJECT | JF_PURE?] (JO_FIELD key)* (JO_OR lit)? (JO_LENGTH | JO_UPPER | JO_REGEX q)?   (at least one of the two)
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
__host__ __device__
#endif
inline bool jmes_chain_form(const uint32_t* p, uint32_t n) {
  if (n < 2 || (p[0] & 0xFFu) != JR_OBJECT) return false;
  uint32_t i = 1;
  while (i + 1 < n && p[i] == JO_FIELD) i += 2;
  bool extra = false;
  if (i + 1 < n && p[i] == JO_OR) { i += 2; extra = true; }
  if (i < n && (p[i] == JO_LENGTH || p[i] == JO_UPPER)) { i += 1; extra = true; }
  else if (i + 1 < n && p[i] == JO_REGEX) { i += 2; extra = true; }
  return extra && i == n;
}
// regex_match precompute (regex.cpp, Batch::str_rx): at most RX_MAX regexes per ruleset (bits 0..RX_MAX-1 of a
// string's word); RX_FB: the string has a byte outside printable ASCII (its pairs go to the CPU engine)
constexpr uint32_t RX_MAX = 31;
constexpr uint32_t RX_FB = 1u << 31;
constexpr uint32_t RX_SYMS = 95;          // DFA alphabet: printable ASCII 0x20..0x7E
constexpr uint32_t RX_MAX_STATES = 1024;
constexpr uint32_t JMES_MAX_LIST = 32;     // virtual list capacity (longer -> CPU fallback)
constexpr uint32_t JMES_KEYBIT = 1u << 31; // virtual list element: the key of map entry node (index & ~KEYBIT)
constexpr uint32_t JMES_SIDBIT = 1u << 30; // virtual list element: a string value, by dictionary id (& ~SIDBIT)
                                           // (compiled kernels: the string came with its path column entry)
enum StrValFlag : uint8_t { SV_LIST = 1, SV_JSON = 2, SV_RANGE = 4 };  // literal string value: json []string ok,
                                                                        // json.Valid, InRange operator pattern
struct CondOperand {     // 16 bytes
  uint8_t kind;          // OperandKind
  uint8_t sv;            // StrValFlag (literal strings)
  uint16_t nseg;         // OK_PATH: path segments
  uint32_t a;            // OK_LIT: cnodes index; OK_PATH: pool offset of the segments' key sids
  uint32_t list, nlist;  // SV_LIST: pool offset / count of the []string element sids; OK_PATH: list = the path
                         // column of the whole path + 1 (0: none), read before the key-by-key search
};
struct Cond {            // 48 bytes
  uint8_t op;            // CondOp
  uint8_t pad[3];
  uint32_t leaf;         // SV_RANGE value: pattern leaf of the value string (handleRange, anyin.go:98-104)
  uint32_t leaf_neg;     // ... and of its first "-" replaced by "!-" (AnyNotIn, anyin.go:143-152)
  uint32_t pad2;
  CondOperand key, value;
};
struct CondProg {        // 16 bytes
  uint32_t any0, nany;   // nany == NONE: no `any` block
  uint32_t all0, nall;
};
static_assert(sizeof(Cond) == 48, "cond size");

enum RuleFlag : uint8_t { RD_GATE_EXACT = 1,    // match == the batch's kind gate (kinds-only filters, no exclude)
                          RD_USES_OPERATION = 2 // a condition reads request.operation (background: "CREATE")
};

// foreach validation (validation.go:319-421), RK_FOREACH: RuleDesc.root = pool offset of [n, entry offsets...];
// an entry is [list operand (pool offset of a CondOperand copy), preconditions CondProg or NONE, deny CondProg,
// elementScope (0 unset, 1 false, 2 true)]
// foreach entry validator (validation.go:276-317 on the element's validator: deny > pattern / anyPattern > foreach)
enum ForeachKind : uint32_t { FE_DENY = 0, FE_PATTERN = 1, FE_ANYPATTERN = 2, FE_NESTED = 3, FE_NONE = 4 };
struct ForeachEntry {
  CondOperand list;
  uint32_t pre, deny, scope;  // scope: 0 unset, 1 false, 2 true
  uint32_t kind;              // ForeachKind
  uint32_t body;              // FE_PATTERN: pattern root; FE_ANYPATTERN: pool offset of the roots; FE_NESTED: pool
                              // offset of the nested entries ([n, entries...], as the rule's own list)
  uint32_t nalts;             // FE_ANYPATTERN: alternatives
  uint32_t dyn;               // pool offset of the element variables of its pattern(s): [n, (kind, nseg, segs...)...]
                              // (kind 0: element path, 1: elementIndex), NONE without any
};

struct RuleDesc {
  uint8_t kind;
  uint8_t uses_meta;     // pattern contains metadata-expansion sites
  uint8_t nslots;
  uint8_t flags;         // RuleFlag
  uint32_t policy;       // policy index
  MatchBlock match, exclude;
  uint32_t empty_may_match;  // evaluate the empty-OldResource retry (validation.go:606)
  uint32_t root;         // RK_PATTERN: root pnode; RK_ANYPATTERN: first of nalts root ids in pool; RK_PSS: PssDesc
  uint32_t nalts;
  uint32_t meta_sites, nmeta;
  uint32_t pre;          // precondition program (CondProg index) or NONE; RK_DENY: `root` is the deny program
  uint32_t exc;          // PolicyException candidates or NONE: pool offset of [n, then (mode, filters, nfilters) per
                         // candidate in FindExceptions order] (compiler.cpp compile_exceptions)
};

// ---------------------------------------------------------------- results
enum Status : uint8_t { ST_NONE = 0, ST_PASS = 1, ST_FAIL = 2, ST_SKIP = 3, ST_ERROR = 4, ST_FALLBACK = 5, ST_PANIC = 6,
                        ST_ND = 7 };
constexpr int NSTATUS = 8;
// high 5 bits of a status byte: the passing anyPattern alternative (ST_PASS), or ST_MARK_PRE on a skip / error that
// came from the rule's preconditions ("preconditions not met", validation.go:286-288)
constexpr uint8_t ST_MARK_PRE = 30u << 3;
// on an error of a foreach rule: an element that is not a map under elementScope: true (validation.go:395-397)
constexpr uint8_t ST_MARK_SCOPE = 29u << 3;
// transient (never returned): a PodSecurity pair pss_kernel left to pss_map_kernel (the map walk: exclusion
// sub-pods, resources without path columns); low bits ST_NONE
constexpr uint8_t ST_PSS_MAP = 28u << 3;
// on a skip: rule skipped due to the PolicyException candidate (mark - 1) of the rule (validation.go:824-848)
constexpr uint32_t MAX_EXC = 27;
// (the status byte is ST_SKIP | (i + 1) << 3 for candidate i < MAX_EXC)

constexpr int MAX_IDX = 4;
constexpr int MAX_SLOTS = 2;
constexpr int MAX_DEPTH = 24;
constexpr int MAX_ALTS = 8;

struct FailRec {        // 32 bytes; one per failing pattern (per failing anyPattern alternative)
  uint32_t res, rule;
  uint32_t tmpl;        // path template (NONE: no path, i.e. "failed: <err>" message)
  uint16_t alt;         // anyPattern alternative (0 for single patterns)
  uint16_t nalt;        // failing alternatives recorded for this pair
  uint16_t idx[MAX_IDX];
  uint32_t key[MAX_SLOTS];
};
static_assert(sizeof(FailRec) == 32, "fail record size");
// A failing-path record as the walk stages it for a rule without metadata-expansion sites (no resolved keys): the
// rule and the match wave are those of the staging chunk, so 16 bytes carry the rest (compact_copy_kernel expands
// it to a FailRec). Rules with expansion sites stage whole FailRecs.
struct StageRec {
  uint32_t tmpl;
  uint32_t lane_alt;    // resource offset in the chunk's match wave (bits 0..5) | alternative << 8
  uint16_t idx[MAX_IDX];
};
static_assert(sizeof(StageRec) == 16, "staged record size");

}  // namespace kyv
