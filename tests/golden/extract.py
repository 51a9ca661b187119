#!/usr/bin/env python3
"""Golden-vector extractor (test infrastructure).

Reads the reference's own Go test sources and YAML fixtures AS TEXT (nothing from the reference is
executed or imported) and writes small JSON fixtures next to this script:

  wildcard.json      pkg/utils/wildcard/match_test.go            (go-wildcard v1.0.3 semantics)
  pattern_leaf.json  pkg/engine/pattern/pattern_test.go           (leaf comparison semantics)
  validate_walk.json pkg/engine/validate/validate_test.go         (pattern walk: paths, skip/pass)
  engine.json        pkg/engine/validation_test.go                (end-to-end statuses + messages)
  pss.json           pkg/pss/evaluate_test.go                     (PSS verdicts)
  cli.json           test/cli/test/*/kyverno-test.yaml + inputs   (CLI `kyverno test` results)
  best_practices.json test/best_practices/*.yaml                  (C1 / C3 policy set)
  chart_restricted.json charts/kyverno-policies/templates/**      (hand-rendered PSS restricted profile)
  conditions.json    pkg/engine/variables/evaluate_test.go        (condition operators: key, operator, value -> bool)
  match.json         pkg/engine/utils_test.go TestMatchesResourceDescription(+_GenerateName) (match / exclude)
  match_units.json   pkg/utils/match/{name,annotations,labels,kind}_test.go, pkg/utils/kube/kind_test.go
  autogen.json       pkg/autogen/autogen_test.go (rule names, CanAutoGen / GetSupportedControllers, rule counts)
  policycache.json   pkg/policycache/cache_test.go (validate lookups by type / kind / namespace)
  anchor.json        pkg/engine/anchor/*_test.go (Parse, String, predicates, error classes, path / map helpers)
  references.json    $() references: validate_test.go reference walks, vars_test.go substitution / absolute paths
  cli_apply.json     cmd/cli/kubectl-kyverno/apply/apply_command_test.go Test_Apply (report summaries of
                     `kyverno apply` over local policy / resource files, incl. test/cli/apply: foreach + JMESPath)

Usage: python tests/golden/extract.py [/root/reference]
"""
import ast
import glob
import json
import os
import re
import sys

import yaml

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def read(p):
    with open(os.path.join(REF, p), encoding="utf-8") as f:
        return f.read()


def write(name, data):
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"{name}: {len(data)} records")


def go_unquote(s):
    """Go interpreted string literal (with quotes) -> str."""
    return ast.literal_eval(s)


def functions(src):
    """split Go source into (name, body) for top-level funcs."""
    out = []
    for m in re.finditer(r"^func (\w+)\(", src, re.M):
        start = m.start()
        nxt = re.search(r"^func \w+\(", src[m.end():], re.M)
        end = m.end() + nxt.start() if nxt else len(src)
        out.append((m.group(1), src[start:end]))
    return out


# ---------------------------------------------------------------- wildcard
def extract_wildcard():
    src = read("pkg/utils/wildcard/match_test.go")
    recs = []
    for m in re.finditer(r'pattern:\s*("(?:[^"\\]|\\.)*"),\s*text:\s*("(?:[^"\\]|\\.)*"),\s*matched:\s*(true|false)', src):
        recs.append({"pattern": go_unquote(m.group(1)), "text": go_unquote(m.group(2)), "matched": m.group(3) == "true"})
    src2 = read("pkg/utils/match/name_test.go") if os.path.exists(os.path.join(REF, "pkg/utils/match/name_test.go")) else ""
    write("wildcard.json", recs)


# ---------------------------------------------------------------- pattern leaf
GO_LIT = r'("(?:[^"\\]|\\.)*"|-?\d+\.\d+|-?\d+|true|false|nil|\w+)'
OPS = {"operator.Equal": "", "operator.NotEqual": "!", "operator.More": ">", "operator.Less": "<",
       "operator.MoreEqual": ">=", "operator.LessEqual": "<="}


def go_value(tok, env):
    if tok.startswith('"'):
        return {"json": json.dumps(go_unquote(tok))}
    if tok in ("true", "false"):
        return {"json": tok}
    if tok == "nil":
        return {"json": "null"}
    if re.fullmatch(r"-?\d+\.\d+", tok):
        return {"json": tok}  # float64 (decimal point kept -> float)
    if re.fullmatch(r"-?\d+", tok):
        return {"json": tok}  # Go int
    if tok in env:
        return env[tok]
    return None


def extract_pattern_leaf():
    src = read("pkg/engine/pattern/pattern_test.go")
    recs = []
    for fname, body in functions(src):
        env = {}
        raws = dict(re.findall(r"(\w+) := \[\]byte\(`(.*?)`\)", body, re.S))
        for line in body.splitlines():
            line = line.strip()
            m = re.match(r'(\w+) :?= ("(?:[^"\\]|\\.)*")$', line)
            if m:
                env[m.group(1)] = {"json": json.dumps(go_unquote(m.group(2)))}
                continue
            m = re.match(r"assert\.Assert\(t, (!?)(\w+)\(logger, (.*)\)\)$", line)
            if not m:
                continue
            neg, fn, args = m.group(1) == "!", m.group(2), m.group(3)
            if fn == "Validate" and 'value["key"]' in args:
                v = json.loads(raws["rawValue"])["key"]
                p = json.loads(raws["rawPattern"])["key"]
                recs.append({"test": fname, "fn": "Validate", "value": json.dumps(v), "value_float": True,
                             "pattern": json.dumps(p), "expect": not neg})
                continue
            toks = [t.strip() for t in re.findall(r'"(?:[^"\\]|\\.)*"|[^,]+', args)]
            toks = [t for t in toks if t]
            if fn in ("Validate", "validateFloatPattern", "validateStringPattern", "validateStringPatterns"):
                v, p = go_value(toks[0], env), go_value(toks[1], env)
                if v is None or p is None:
                    continue
                recs.append({"test": fname, "fn": fn, "value": v["json"], "pattern": p["json"], "expect": not neg})
            elif fn == "validateNilPattern":
                v = go_value(toks[0], env)
                recs.append({"test": fname, "fn": fn, "value": v["json"], "pattern": "null", "expect": not neg})
            elif fn in ("validateString", "compareString"):
                v, p = go_value(toks[0], env), go_value(toks[1], env)
                op = OPS[toks[2]]
                recs.append({"test": fname, "fn": fn, "value": v["json"], "pattern": p["json"], "op": op, "expect": not neg})
    write("pattern_leaf.json", recs)


# ---------------------------------------------------------------- validate walk
def extract_validate_walk():
    src = read("pkg/engine/validate/validate_test.go")
    recs = []
    for fname, body in functions(src):
        if fname.startswith("testMatchPattern"):
            continue
        if "testCases := []struct" in body:
            for m in re.finditer(r'name:\s*"([^"]*)",\s*pattern:\s*\[\]byte\(`(.*?)`\),\s*resource:\s*\[\]byte\(`(.*?)`\),\s*status:\s*engineapi\.RuleStatus(\w+)', body, re.S):
                recs.append({"test": f"{fname}/{m.group(1)}", "entry": "MatchPattern", "pattern": m.group(2),
                             "resource": m.group(3), "status": m.group(4).lower()})
            continue
        if "SubstituteAll" in body or "$(" in body:
            continue  # reference/variable tests -> CPU fallback path, not the GPU walk
        raws = dict(re.findall(r"(\w+) := \[\]byte\(`(.*?)`\)", body, re.S))
        if "rawPattern" not in raws:
            continue
        res_key = next((k for k in ("rawMap", "rawResource", "rawArray") if k in raws), None)
        if res_key is None:
            continue
        call = re.search(r"(validateMap|validateResourceElement|validateArray|MatchPattern)\(", body)
        if not call:
            continue
        mpath = re.search(r'assert\.Equal\(t, path, "([^"]*)"\)', body)
        errnil = None
        if re.search(r"assert\.Assert\(t, err != nil\)", body):
            errnil = False
        elif re.search(r"assert\.(NilError\(t, err\)|Assert\(t, err == nil\))", body[call.start():]):
            errnil = True
        recs.append({"test": fname, "entry": call.group(1), "pattern": raws["rawPattern"], "resource": raws[res_key],
                     "path": mpath.group(1) if mpath else None, "err_nil": errnil})
    write("validate_walk.json", recs)


# ---------------------------------------------------------------- engine (validation_test.go)
def extract_engine():
    src = read("pkg/engine/validation_test.go")
    recs = []
    for fname, body in functions(src):
        raws = dict(re.findall(r"(\w+) := \[\]byte\(`(.*?)`\)", body, re.S))
        if "policyRaw" in raws and "resourceRaw" in raws and "rawPolicy" not in raws:  # deny-condition tests
            raws["rawPolicy"], raws["rawResource"] = raws["policyRaw"], raws["resourceRaw"]
        if "rawPolicy" in raws and "rawResource" in raws and "testCases" not in body:
            m = re.search(r"msgs := \[\]string\{(.*?)\}\n", body, re.S)
            msgs = [go_unquote(x) for x in re.findall(r'"(?:[^"\\]|\\.)*"', m.group(1))] if m else None
            succ = None
            if re.search(r"assert\.Assert\(t, !er\.IsSuccessful\(\)\)", body):
                succ = False
            elif re.search(r"assert\.Assert\(t, er\.IsSuccessful\(\)\)", body):
                succ = True
            if msgs is None and succ is None:
                continue
            recs.append({"test": fname, "policy": raws["rawPolicy"], "resource": raws["rawResource"],
                         "msgs": msgs, "successful": succ})
        elif "expectedResults" in body and "expectedMessages" in body:  # Test_Flux_Kustomization_PathNotPresent
            for m in re.finditer(r'name:\s*"([^"]*)",\s*policyRaw:\s*\[\]byte\(`(.*?)`\),.*?resourceRaw:\s*\[\]byte\(`(.*?)`\),'
                                 r'\s*expectedResults:\s*\[\]engineapi\.RuleStatus\{(.*?)\},\s*expectedMessages:\s*\[\]string\{(.*?)\},\n',
                                 body, re.S):
                sts = [x.replace("RuleStatus", "").lower() for x in re.findall(r"engineapi\.(\w+)", m.group(4))]
                msgs = [go_unquote(x) for x in re.findall(r'"(?:[^"\\]|\\.)*"', m.group(5))]
                recs.append({"test": f"{fname}/{m.group(1)}", "policy": m.group(2), "resource": m.group(3),
                             "msgs": msgs, "statuses": sts})
        elif "testCases" in body and "expectedFailed" in body:
            pol = raws.get("rawPolicy")
            for m in re.finditer(r'description:\s*"([^"]*)",\s*rawPolicy:\s*(\w+),\s*rawResource:\s*\[\]byte\(`(.*?)`\),\s*expected(\w+):\s*true', body, re.S):
                recs.append({"test": f"{fname}/{m.group(1)}", "policy": raws.get(m.group(2), pol), "resource": m.group(3),
                             "msgs": None, "expect": m.group(4).lower()})
    write("engine.json", recs)


# ---------------------------------------------------------------- PSS
def extract_pss():
    src = read("pkg/pss/evaluate_test.go")
    recs = []
    for m in re.finditer(r'name:\s*"([^"]*)",\s*rawRule:\s*\[\]byte\(`(.*?)`\),\s*rawPod:\s*\[\]byte\(`(.*?)`\),\s*allowed:\s*(true|false)', src, re.S):
        recs.append({"name": m.group(1), "rule": m.group(2), "pod": m.group(3), "allowed": m.group(4) == "true"})
    write("pss.json", recs)


# ---------------------------------------------------------------- YAML helpers
def yaml_docs(path):
    with open(path, encoding="utf-8") as f:
        return [d for d in yaml.safe_load_all(f) if d is not None]


def normalize_numbers(x):
    """sigs.k8s.io/yaml converts YAML to JSON through json.Marshal: integral float64 values < 1e21 are
    written without a fraction and then decode as int64 in unstructured objects."""
    if isinstance(x, dict):
        return {str(k): normalize_numbers(v) for k, v in x.items()}
    if isinstance(x, list):
        return [normalize_numbers(v) for v in x]
    if isinstance(x, float) and x == int(x) and abs(x) < 1e21:
        return int(x)
    return x


def json_safe(x):
    return json.loads(json.dumps(x, default=str))


# ---------------------------------------------------------------- CLI goldens
def extract_cli():
    recs = []
    for d in sorted(glob.glob(os.path.join(REF, "test/cli/test/*"))):
        kt = os.path.join(d, "kyverno-test.yaml")
        if not os.path.exists(kt):
            continue
        try:
            spec = yaml_docs(kt)[0]
        except Exception:
            continue
        if spec.get("variables") or spec.get("userinfo"):
            continue
        policies, resources = [], []
        ok = True
        for p in spec.get("policies", []):
            fp = os.path.join(d, p)
            if not os.path.exists(fp):
                ok = False
                break
            policies += [json_safe(x) for x in yaml_docs(fp)]
        for r in spec.get("resources", []):
            fp = os.path.join(d, r)
            if not os.path.exists(fp):
                ok = False
                break
            resources += [json_safe(normalize_numbers(x)) for x in yaml_docs(fp)]
        if not ok:
            continue
        results = []
        for res in spec.get("results", []):
            names = res.get("resources") or ([res["resource"]] if res.get("resource") else [])
            for n in names:
                results.append({"policy": res.get("policy"), "rule": res.get("rule"), "resource": n,
                                "kind": res.get("kind"), "result": res.get("result") or res.get("status"),
                                "namespace": res.get("namespace")})
        recs.append({"dir": os.path.basename(d), "policies": policies, "resources": resources, "results": results})
    write("cli.json", recs)


def extract_best_practices():
    recs = []
    for p in sorted(glob.glob(os.path.join(REF, "test/best_practices/*.yaml"))):
        for doc in yaml_docs(p):
            if isinstance(doc, dict) and doc.get("kind") in ("ClusterPolicy", "Policy"):
                recs.append({"file": os.path.basename(p), "policy": json_safe(doc)})
    write("best_practices.json", recs)


# ---------------------------------------------------------------- chart (hand-rendered)
def render_chart_template(text, name, level):
    """Render charts/kyverno-policies templates with values.yaml defaults (podSecurityStandard=<level>,
    validationFailureAction=audit, background=true, failurePolicy=Fail, no excludes/preconditions,
    autogenControllers empty). Only the constructs these templates use are handled."""
    def cond(expr):
        expr = expr.strip()
        if expr.startswith("with"):
            return False  # every `with` reads an empty value (excludes, overrides, autogenControllers, ...)
        if expr.startswith("if eq (include"):
            return True  # the policy is part of the selected profile
        if expr.startswith("if .Values.podSecuritySeverity"):
            return True
        return False  # $preconditionsN, .all: empty

    out = []
    stack = []  # list of [active_now, parent_active, taken]
    active = True
    for line in text.splitlines():
        s = line.strip()
        m = re.fullmatch(r"\{\{-?\s*(.*?)\s*-?\}\}", s)
        if m and not s.startswith("{{`"):
            d = m.group(1)
            if d.startswith("if ") or d.startswith("with "):
                c = cond(d)
                stack.append([active, c])
                active = active and c
            elif d.startswith("else"):
                parent, c = stack[-1]
                stack[-1][1] = not c
                active = parent and not c
            elif d.startswith("end"):
                parent, _ = stack.pop()
                active = parent
            continue  # $name :=, include, toYaml ... lines produce nothing with empty values
        if not active:
            continue
        if "labels: {{ include" in line:
            continue
        line = line.replace("{{ $name }}", name)
        line = line.replace("{{ .Values.background }}", "true")
        line = line.replace("{{ .Values.failurePolicy }}", "Fail")
        line = line.replace("{{ .Values.validationFailureAction }}", "audit")
        line = line.replace("{{ .Values.podSecuritySeverity | quote }}", '"medium"')
        line = line.replace("{{ .Values.podSecuritySeverity }}", "medium")
        line = line.replace("{{`{{`}}", "{{").replace("{{`}}`}}", "}}")
        line = re.sub(r"\{\{`(.*?)`\}\}", r"\1", line)
        out.append(line)
    return yaml.safe_load("\n".join(out))


def extract_chart():
    recs = []
    base = os.path.join(REF, "charts/kyverno-policies/templates")
    for level_dir in ("baseline", "restricted"):
        for p in sorted(glob.glob(os.path.join(base, level_dir, "*.yaml"))):
            text = open(p, encoding="utf-8").read()
            name = re.search(r'\$name := "([^"]+)"', text).group(1)
            doc = render_chart_template(text, name, "restricted")
            recs.append({"file": f"{level_dir}/{os.path.basename(p)}", "policy": json_safe(doc)})
    write("chart_restricted.json", recs)


# ---------------------------------------------------------------- condition operators
class _GoLit:
    """Tiny parser for the Go composite literals used as condition keys/values in evaluate_test.go:
    strings, ints, floats, int64(..), bools, nil, []interface{}{...}, []string{...}, map[string]interface{}{k: v}."""

    def __init__(self, s):
        self.s, self.i = s, 0

    def ws(self):
        while self.i < len(self.s) and self.s[self.i] in " \t\n,":
            self.i += 1

    def parse(self):
        self.ws()
        s, i = self.s, self.i
        if s[i] == '"':
            m = re.match(r'"(?:[^"\\]|\\.)*"', s[i:])
            self.i += m.end()
            return ("str", go_unquote(m.group(0)))
        if s.startswith("[]", i):
            self.i += re.match(r"\[\](?:interface\{\}|[\w.\[\]]+)\{", s[i:]).end()
            items = []
            while True:
                self.ws()
                if s[self.i] == "}":
                    self.i += 1
                    return ("arr", items)
                items.append(self.parse())
        if s.startswith("map[", i):
            self.i += re.match(r"map\[\w+\](?:interface\{\}|\w+)\{", s[i:]).end()
            items = []
            while True:
                self.ws()
                if s[self.i] == "}":
                    self.i += 1
                    return ("map", items)
                k = self.parse()
                self.ws()
                assert s[self.i] == ":"
                self.i += 1
                items.append((k[1], self.parse()))
        m = re.match(r"(int64|float64|int)\(([^()]*)\)", s[i:])
        if m:
            self.i += m.end()
            return ("num", m.group(2).strip(), m.group(1) == "float64")
        m = re.match(r"true|false|nil", s[i:])
        if m:
            self.i += m.end()
            return ("lit", m.group(0))
        m = re.match(r"-?[0-9][0-9.eE+-]*", s[i:])
        self.i += m.end()
        return ("num", m.group(0), "." in m.group(0) or "e" in m.group(0).lower())


def _go_marshal(v):
    """json.Marshal of the decoded Go value (encoding/json: float64 integral values print without fraction)."""
    t = v[0]
    if t == "str":
        return json.dumps(v[1])
    if t == "lit":
        return "null" if v[1] == "nil" else v[1]
    if t == "num":
        if v[2]:
            f = float(v[1])
            return str(int(f)) if f == int(f) and abs(f) < 1e21 else repr(f)
        return str(int(v[1]))
    if t == "arr":
        return "[" + ",".join(_go_marshal(x) for x in v[1]) + "]"
    return "{" + ",".join(json.dumps(k) + ":" + _go_marshal(x) for k, x in sorted(v[1])) + "}"


def extract_conditions():
    src = read("pkg/engine/variables/evaluate_test.go")
    body = dict(functions(src))["TestEvaluate"]
    recs = []
    pat = re.compile(r'\{kyverno\.Condition\{RawKey: kyverno\.ToJSON\((.*?)\), Operator: kyverno\.ConditionOperators\["(\w+)"\], '
                     r'RawValue: kyverno\.ToJSON\((.*?)\)\}, (true|false)\},\s*$')
    for ln, line in enumerate(body.splitlines()):
        m = pat.search(line.strip())
        if not m:
            continue
        key, op, val, want = m.groups()
        recs.append({"key": _go_marshal(_GoLit(key).parse()), "operator": op,
                     "value": _go_marshal(_GoLit(val).parse()), "result": want == "true",
                     "src": "pkg/engine/variables/evaluate_test.go TestEvaluate #%d" % len(recs)})
    write("conditions.json", recs)


# ---------------------------------------------------------------- match / exclude (MatchesResourceDescription)
def extract_match():
    """pkg/engine/utils_test.go TestMatchesResourceDescription + _GenerateName: (policy JSON, resource JSON, whether
    MatchesResourceDescription returns an error for every autogen-computed rule); the admission info of each case
    is kept as text (it only matters for rules naming roles / clusterRoles / subjects)."""
    src = read("pkg/engine/utils_test.go")
    fns = dict(functions(src))
    recs = []
    for fn in ("TestMatchesResourceDescription", "TestMatchesResourceDescription_GenerateName"):
        body = fns[fn]
        for blk in re.split(r"\n\t\t\{\n\t\t\tDescription:", body)[1:]:
            desc = re.match(r'\s*"((?:[^"\\]|\\.)*)"', blk).group(1)
            res = re.search(r"Resource:\s*\[\]byte\(`(.*?)`\)", blk, re.S).group(1)
            pol = re.search(r"Policy:\s*\[\]byte\(`(.*?)`\)", blk, re.S).group(1)
            err = re.search(r"areErrorsExpected:\s*(true|false)", blk).group(1) == "true"
            adm = re.search(r"AdmissionInfo:\s*v1beta1\.RequestInfo\{(.*?)\n\t\t\t\},", blk, re.S)
            recs.append({"test": fn, "description": desc, "resource": json.loads(res), "policy": json.loads(pol),
                         "errors_expected": err, "admission_info": adm.group(1).strip() if adm else ""})
    write("match.json", recs)


# ---------------------------------------------------------------- Go composite literals (table tests)
class _GoExpr:
    """Go composite-literal expressions of table-driven tests -> Python values: strings, numbers, true/false/nil,
    [&]Type{...} (keyed elements -> dict, positional -> list), map[..]..{k: v}, qualified constants (kept as
    their name, e.g. "metav1.LabelSelectorOpIn")."""

    def __init__(self, s):
        self.s, self.i = s, 0

    def ws(self):
        while self.i < len(self.s) and self.s[self.i] in " \t\n\r,":
            self.i += 1
        while self.s.startswith("//", self.i):
            self.i = self.s.index("\n", self.i)
            self.ws()

    def value(self):
        self.ws()
        s, i = self.s, self.i
        if s[i] == '"':
            m = re.match(r'"(?:[^"\\]|\\.)*"', s[i:])
            self.i += m.end()
            return go_unquote(m.group(0))
        if s[i] == "`":
            j = s.index("`", i + 1)
            self.i = j + 1
            return s[i + 1:j]
        if s[i] == "{":  # untyped composite (element of a typed slice)
            return self.composite()
        if s[i] == "&":
            self.i += 1
            return self.value()
        m = re.match(r"(map\[[^\]]*\](?:interface\{\}|[\w.*\[\]])*|\[\](?:interface\{\}|[\w.*\[\]])*|[A-Za-z_][\w.]*)\{",
                     s[i:])
        if m:
            self.i += m.end() - 1
            return self.composite()
        m = re.match(r"true|false|nil", s[i:])
        if m:
            self.i += m.end()
            return {"true": True, "false": False, "nil": None}[m.group(0)]
        m = re.match(r"-?[0-9][0-9.eE+-]*", s[i:])
        if m:
            self.i += m.end()
            t = m.group(0)
            return float(t) if any(c in t for c in ".eE") else int(t)
        m = re.match(r"[A-Za-z_][\w.]*", s[i:])
        self.i += m.end()
        return m.group(0)

    def composite(self):
        assert self.s[self.i] == "{"
        self.i += 1
        keyed, items = {}, []
        while True:
            self.ws()
            if self.s[self.i] == "}":
                self.i += 1
                return keyed if keyed else items
            v = self.value()
            self.ws()
            if self.s[self.i] == ":":
                self.i += 1
                keyed[v] = self.value()
            else:
                items.append(v)


def _go_table(body):
    """the composite literal of `tests := []struct{...}{...}` (or `tcs`) -> list of dicts"""
    m = re.search(r"(?:tests|tcs|testcases)\s*:?=\s*\[\]struct\s*\{", body)
    i = m.end()
    depth = 1
    while depth:  # skip the struct type
        depth += {"{": 1, "}": -1}.get(body[i], 0)
        i += 1
    g = _GoExpr(body[i:])
    return g.composite()


def _selector_json(sel):
    if sel is None:
        return None
    if isinstance(sel, list):  # &metav1.LabelSelector{}
        sel = {}
    out = {}
    if sel.get("MatchLabels") is not None:
        out["matchLabels"] = sel["MatchLabels"]
    if sel.get("MatchExpressions") is not None:
        ops = {"metav1.LabelSelectorOpIn": "In", "metav1.LabelSelectorOpNotIn": "NotIn",
               "metav1.LabelSelectorOpExists": "Exists", "metav1.LabelSelectorOpDoesNotExist": "DoesNotExist"}
        out["matchExpressions"] = [{"key": e.get("Key", ""), "operator": ops.get(e.get("Operator"), e.get("Operator")),
                                    "values": e.get("Values")} for e in sel["MatchExpressions"]]
    return out


def extract_match_units():
    """pkg/utils/match/{name,annotations,labels,kind}_test.go and pkg/utils/kube/kind_test.go"""
    out = {}
    src = read("pkg/utils/match/name_test.go")
    out["name"] = [{"expected": (t.get("args") or {}).get("expected", ""), "actual": (t.get("args") or {}).get("actual", ""),
                    "want": t["want"]} for t in _go_table(dict(functions(src))["TestCheckName"])]
    src = read("pkg/utils/match/annotations_test.go")
    out["annotations"] = [{"expected": t["args"].get("expected") or {}, "actual": t["args"].get("actual") or {},
                           "want": t["want"]} for t in _go_table(dict(functions(src))["TestCheckAnnotations"])]
    src = read("pkg/utils/match/labels_test.go")
    out["selector"] = [{"expected": _selector_json(t["args"].get("expected")), "actual": t["args"].get("actual") or {},
                        "want": t.get("want", False), "wantErr": t.get("wantErr", False)}
                       for t in _go_table(dict(functions(src))["TestCheckSelector"])]
    src = read("pkg/utils/match/kind_test.go")
    kinds = []
    pat = re.compile(r'CheckKind\(subresourceGVKToAPIResource, \[\]string\{"([^"]*)"\}, schema\.GroupVersionKind\{Kind: "([^"]*)", '
                     r'Group: "([^"]*)", Version: "([^"]*)"\}, "([^"]*)", (true|false)\)\s*assert\.Equal\(t, match, (true|false)\)', re.S)
    subres_map = False
    for m in pat.finditer(src):
        before = src[:m.start()]
        subres_map = "subresourceGVKToAPIResource[" in before
        kinds.append({"kinds": [m.group(1)], "kind": m.group(2), "group": m.group(3), "version": m.group(4),
                      "subresource": m.group(5), "allow_ephemeral": m.group(6) == "true", "want": m.group(7) == "true",
                      "subresource_map": subres_map})
    out["check_kind"] = kinds
    src = read("pkg/utils/kube/kind_test.go")
    out["gvk"] = [{"gvk": a, "group_version": b, "kind": c} for a, b, c in re.findall(
        r'apiVersion, kind = GetKindFromGVK\("([^"]*)"\)\s*assert\.Equal\(t, "([^"]*)", apiVersion\)\s*'
        r'assert\.Equal\(t, "([^"]*)", kind\)', src)]
    out["gv_matches"] = [{"group_version": a, "server": b, "want": c == "true"} for a, b, c in re.findall(
        r'groupVersion, serverResourceGroupVersion :?= "([^"]*)", "([^"]*)"\s*(?://[^\n]*\s*)?'
        r'assert\.Equal\(t, GroupVersionMatches\(groupVersion, serverResourceGroupVersion\), (true|false)\)', src)]
    write("match_units.json", out)


# ---------------------------------------------------------------- autogen
def extract_autogen():
    """pkg/autogen/autogen_test.go: getAutogenRuleName (name truncation), CanAutoGen / GetSupportedControllers
    tables (policy JSON -> "none" or the pod controllers), Test_PodSecurityWithNoExceptions (3 computed rules)"""
    src = read("pkg/autogen/autogen_test.go")
    fns = dict(functions(src))
    out = {"rule_names": [], "controllers": [], "rule_counts": []}
    for name, rule, prefix, exp in re.findall(r'\{"([^"]*)", "([^"]*)", "([^"]*)", "([^"]*)"\}', fns["Test_getAutogenRuleName"]):
        out["rule_names"].append({"rule": rule, "prefix": prefix, "expected": exp})
    for fn in ("Test_CanAutoGen", "Test_GetSupportedControllers"):
        for m in re.finditer(r'name:\s*"([^"]*)",\s*policy:\s*\[\]byte\(`(.*?)`\),\s*expectedControllers:\s*("[^"]*"|PodControllers)',
                             fns[fn], re.S):
            exp = m.group(3)
            out["controllers"].append({"test": fn, "name": m.group(1), "policy": json.loads(m.group(2)),
                                       "controllers": "pod" if exp == "PodControllers" else go_unquote(exp)})
    m = re.search(r"policy := \[\]byte\(`(.*?)`\).*?assert\.Equal\(t, (\d+), len\(rules\)\)",
                  fns["Test_PodSecurityWithNoExceptions"], re.S)
    out["rule_counts"].append({"policy": json.loads(m.group(1)), "rules": int(m.group(2))})
    write("autogen.json", out)


# ---------------------------------------------------------------- anchor package unit tables
def extract_anchor():
    """pkg/engine/anchor/{anchor,error,utils,anchormap}_test.go: Parse, New / String / Type / Key, the Is*
    predicates, the anchor-error classifiers, RemoveAnchorsFromPath, GetAnchorsResourcesFromMap,
    resourceHasValueForKey and AnchorMap.KeysAreMissing, as (op, inputs, want) records"""
    out = []
    src = read("pkg/engine/anchor/anchor_test.go")
    fns = dict(functions(src))
    LQ = r'"(?:[^"\\]|\\.)*"'
    lit = "(" + LQ + ")"
    anc = r"(nil|anchor\{\w+, " + LQ + r"\})"

    def anchor_want(want):
        if want == "nil":
            return None
        t, k = re.match(r"anchor\{(\w+), (" + LQ + r")\}", want).groups()
        return {"type": t, "key": go_unquote(k)}

    for a, want in re.findall(r"args: args\{" + lit + r"\},\s*want: " + anc, fns["TestParse"]):
        out.append({"test": "TestParse", "op": "parse", "a": go_unquote(a), "want": anchor_want(want)})
    for t, k, want in re.findall(r"args: args\{(\w+), " + lit + r"\},\s*want: " + lit, fns["TestString"]):
        out.append({"test": "TestString", "op": "string", "a": t, "b": go_unquote(k), "want": go_unquote(want)})
    for t, k, want in re.findall(r"fields: fields\{(\w+), " + lit + r"\},\s*want: +" + lit, fns["Test_anchor_String"]):
        out.append({"test": "Test_anchor_String", "op": "string", "a": t, "b": go_unquote(k), "want": go_unquote(want)})
    for t, k, want in re.findall(r"args: args\{(\w+), " + lit + r"\},\s*want: " + anc, fns["TestNew"]):
        out.append({"test": "TestNew", "op": "new", "a": t, "b": go_unquote(k), "want": anchor_want(want)})
    for name in ("Test_anchor_Type", "Test_anchor_Key"):
        for t, k, want in re.findall(r"fields: fields\{(\w+), " + lit + r"\},\s*want: +(\w+|" + LQ + r")", fns[name]):
            w = {"type": t, "key": go_unquote(k)}
            out.append({"test": name, "op": "new", "a": t, "b": go_unquote(k), "want": w,
                        "field": want if name.endswith("Type") else go_unquote(want)})
    for name, body in fns.items():
        m = re.match(r"Test(Is\w+|ContainsCondition)$", name)
        if not m or name == "TestIsOneOf":
            continue
        for arg, want in re.findall(r"args: args\{(nil|New\(\w+, " + LQ + r"\))\},\s*want: (true|false)", body):
            t = "" if arg == "nil" else re.match(r"New\((\w+),", arg).group(1)
            out.append({"test": name, "op": "is", "a": m.group(1), "b": t, "want": want == "true"})
    esrc = read("pkg/engine/anchor/error_test.go")
    prefix = {"Negation": ("negation", 2, "negation anchor matched in resource"),
              "Conditional": ("conditional", 0, "conditional anchor mismatch"),
              "Global": ("global", 1, "global anchor mismatch")}
    for name, body in functions(esrc):
        m = re.match(r"TestIs(\w+)AnchorError$", name)
        if not m:
            continue
        kind = prefix[m.group(1)][0]
        for err, want in re.findall(r"err: (nil|errors\.New\(" + LQ + r"\)|new\w+AnchorError\(" + LQ + r"\)),\s*\},\s*want: (true|false)",
                                    body):
            e = None
            mm = re.match(r'errors\.New\((".*")\)', err)
            if mm:
                e = {"code": -1, "msg": go_unquote(mm.group(1))}
            mm = re.match(r'new(\w+)AnchorError\((".*")\)', err)
            if mm:
                _, code, pre = prefix[mm.group(1)]
                e = {"code": code, "msg": pre + ": " + go_unquote(mm.group(2))}
            out.append({"test": name, "op": "err", "a": kind, "b": e, "want": want == "true"})
    usrc = read("pkg/engine/anchor/utils_test.go")
    ufns = dict(functions(usrc))
    for a, want in re.findall(r"str: +" + lit + r",\s*want: " + lit, ufns["TestRemoveAnchorsFromPath"]):
        out.append({"test": "TestRemoveAnchorsFromPath", "op": "remove_path", "a": go_unquote(a), "want": go_unquote(want)})
    body = ufns["TestGetAnchorsResourcesFromMap"]
    for case in re.split(r"\}, \{", body[body.index("}{{") + 3:body.index("for _, tt")]):
        vals = {}
        for fld in ("patternMap", "wantAnchors", "wantResources"):
            i = case.index(fld + ":") + len(fld) + 1
            vals[fld] = _GoExpr(case[i:]).value()
        out.append({"test": "TestGetAnchorsResourcesFromMap", "op": "split", "a": vals["patternMap"],
                    "want": {"anchors": sorted(vals["wantAnchors"]), "resources": sorted(vals["wantResources"])}})
    body = ufns["Test_resourceHasValueForKey"]
    for case in re.split(r"\}, \{", body[body.index("}{{") + 3:body.index("for _, tt")]):
        i = case.index("resource:") + len("resource:")
        g = _GoExpr(case[i:])
        res = g.value()
        key = go_unquote(re.search(r"key: +" + lit, case).group(1))
        want = re.search(r"want: (true|false)", case).group(1) == "true"
        out.append({"test": "Test_resourceHasValueForKey", "op": "has_value", "a": res, "b": key, "want": want})
    body = dict(functions(read("pkg/engine/anchor/anchormap_test.go")))["TestAnchorMap_KeysAreMissing"]
    for case in re.split(r"\}, \{", body[body.index("}{{") + 3:body.index("for _, tt")]):
        i = case.index("anchorMap:") + len("anchorMap:")
        m = _GoExpr(case[i:]).value()
        want = re.search(r"want: (true|false)", case).group(1) == "true"
        out.append({"test": "TestAnchorMap_KeysAreMissing", "op": "keys_missing", "a": m or {}, "want": want})
    write("anchor.json", out)


# ---------------------------------------------------------------- $() references
def extract_references():
    """$() references: pkg/engine/validate/validate_test.go reference cases (pattern, resource, whether the test
    substitutes first, expected walk path / error), pkg/engine/variables/vars_test.go Test_*ReferenceSubstitution
    (document -> expected document) and TestFormAbsolutePath_* (reference, absolute path -> result)"""
    out = []
    for fname, body in functions(read("pkg/engine/validate/validate_test.go")):
        if "$(" not in body:
            continue
        raws = dict(re.findall(r"(\w+) := \[\]byte\(`(.*?)`\)", body, re.S))
        mpath = re.search(r'assert\.Equal\(t, path, "([^"]*)"\)', body)
        errnil = None
        tail = body[body.index("validateResourceElement("):]
        if re.search(r"assert\.Assert\(t, err != nil\)", tail):
            errnil = False
        elif re.search(r"assert\.(NilError\(t, err\)|Assert\(t, err == nil\))", tail):
            errnil = True
        out.append({"test": fname, "kind": "walk", "pattern": json.loads(raws["rawPattern"]),
                    "resource": json.loads(raws["rawMap"]), "substitute": "SubstituteAll" in body,
                    "path": mpath.group(1) if mpath else None, "err_nil": errnil})
    vsrc = read("pkg/engine/variables/vars_test.go")
    for fname, body in functions(vsrc):
        if fname in ("Test_ReferenceSubstitution", "Test_EscpReferenceSubstitution"):
            raws = dict(re.findall(r"(\w+) := \[\]byte\(`(.*?)`\)", body, re.S))
            out.append({"test": fname, "kind": "subst", "document": json.loads(raws["jsonRaw"]),
                        "expected": json.loads(raws["expectedJSON"])})
        elif fname.startswith("TestFormAbsolutePath_"):
            vals = dict(re.findall(r'(\w+) := ("(?:[^"\\]|\\.)*")', body))
            want = vals.get("expectedString")
            if want is None:
                want = vals["referencePath"] if "result == referencePath" in body else vals["absolutePath"]
            out.append({"test": fname, "kind": "abs", "ref": go_unquote(vals["referencePath"]),
                        "at": go_unquote(vals["absolutePath"]), "want": go_unquote(want)})
    write("references.json", out)


# ---------------------------------------------------------------- policy cache
def extract_policycache():
    """pkg/policycache/cache_test.go: the policies of the new*Policy builders, and for every test the validate-type
    lookups (store.get / cache.GetPolicies of ValidateEnforce / ValidateAudit) asserted before the first removal"""
    src = read("pkg/policycache/cache_test.go")
    fns = dict(functions(src))
    builders = {}
    for name, body in fns.items():
        m = re.search(r"rawPolicy := \[\]byte\(`(.*?)`\).*?var policy \*kyvernov1\.(\w+)", body, re.S)
        if name.startswith("new") and m:
            doc = json.loads(m.group(1))
            doc["kind"] = m.group(2)
            builders[name] = doc
    tests = []
    for name, body in fns.items():
        if not name.startswith("Test_"):
            continue
        body = body.split("unsetPolicy(")[0]
        vars_ = dict(re.findall(r"(\w+) := (new\w+)\(t\)", body))
        added = [v for v in re.findall(r"setPolicy\(pCache, (\w+)\)", body)]
        added += [v for v in re.findall(r"cache\.Set\(\w+, (\w+), ", body)]
        if not added:
            continue
        pols = []
        for v in added:
            if v in vars_ and vars_[v] not in pols:
                pols.append(vars_[v])
        nspace = None
        m = re.search(r"nspace := (\w+)\.GetNamespace\(\)", body)
        if m and m.group(1) in vars_:
            nspace = (builders[vars_[m.group(1)]].get("metadata") or {}).get("namespace", "")
        calls = []
        for var, api, typ, kind, ns, rest in re.findall(
                r"(\w+) :?= (pCache\.get|cache\.GetPolicies)\((Validate\w+), \"([^\"]*)\", (\"[^\"]*\"|nspace)\)(.*?)(?=\n\t\w+ :?= |\Z)",
                body, re.S):
            m = re.search(r"if len\(" + var + r"\) != (\d+)", rest)
            if not m:
                continue
            calls.append({"api": "GetPolicies" if api == "cache.GetPolicies" else "get", "type": typ, "kind": kind,
                          "namespace": nspace if ns == "nspace" else go_unquote(ns), "expected": int(m.group(1))})
        if calls:
            tests.append({"test": name, "policies": [builders[b] for b in pols], "calls": calls})
    write("policycache.json", tests)


# ---------------------------------------------------------------- CLI apply summaries
def extract_cli_apply():
    """Test_Apply cases whose policy and resource paths are files of the reference tree: the policies, the
    resources (CLI default namespace applied by the consumer) and the expected report summary."""
    src = read("cmd/cli/kubectl-kyverno/apply/apply_command_test.go")
    body = dict(functions(src))["Test_Apply"]
    local = re.search(r'copyFileToThisDir\("([^"]+)"\)', body).group(1)
    recs = []
    for blk in re.split(r"\n\t\t\{\n\t\t\tconfig: ApplyCommandConfig\{", body)[1:]:
        def paths(key):
            m = re.search(key + r":\s*\[\]string\{([^}]*)\}", blk)
            return re.findall(r'"([^"]*)"', m.group(1)) if m else []
        pols = [p for p in paths("PolicyPaths")] or (["localFileName"] if "localFileName" in blk else [])
        if re.search(r"PolicyPaths:\s*\[\]string\{localFileName\}", blk):
            pols = [local]
        ress = paths("ResourcePaths")
        stdin = re.search(r'stdinFile:\s*"([^"]+)"', blk)
        pols = [stdin.group(1) if (x == "-" and stdin) else x for x in pols]
        ress = [stdin.group(1) if (x == "-" and stdin) else x for x in ress]
        if any(x.startswith("http") for x in pols + ress):
            continue
        summ = {k.lower(): int(v) for k, v in re.findall(r"(Pass|Fail|Skip|Error|Warn):\s*(\d+)", blk)}
        def load(rel):
            fp = os.path.normpath(os.path.join(REF, "cmd/cli/kubectl-kyverno/apply", rel))
            files = sorted(glob.glob(os.path.join(fp, "*.yaml"))) if os.path.isdir(fp) else [fp]
            out = []
            for f in files:
                out += [json_safe(normalize_numbers(x)) for x in yaml_docs(f)]
            return out, [os.path.relpath(f, REF) for f in files]
        policies, pfiles, resources, rfiles = [], [], [], []
        for x in pols:
            d, f = load(x)
            policies += d
            pfiles += f
        for x in ress:
            d, f = load(x)
            resources += d
            rfiles += f
        recs.append({"policy_files": pfiles, "resource_files": rfiles, "policies": policies, "resources": resources,
                     "audit_warn": "AuditWarn:     true" in blk or re.search(r"AuditWarn:\s*true", blk) is not None,
                     "summary": summ})
    write("cli_apply.json", recs)


if __name__ == "__main__" and len(sys.argv) > 2:  # python extract.py <reference> <extractor> ...: selected only
    for name in sys.argv[2:]:
        globals()["extract_" + name]()
    sys.exit(0)

if __name__ == "__main__":
    extract_wildcard()
    extract_pattern_leaf()
    extract_validate_walk()
    extract_engine()
    extract_pss()
    extract_cli()
    extract_best_practices()
    extract_chart()
    extract_conditions()
    extract_cli_apply()
    extract_match()
    extract_match_units()
    extract_autogen()
    extract_policycache()
    extract_anchor()
    extract_references()
