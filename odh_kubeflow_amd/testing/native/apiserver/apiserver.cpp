// odh-apiserver: native (C++) Kubernetes API server for the notebook control plane.
//
// The envtest substitute of SURVEY §7.2 step 2, written natively so that the control
// plane can scale out: the kf / odh managers, the admission webhook replicas and the
// MI355X node agents (one process per GPU) all talk REST + watch to it concurrently.
// Semantics follow odh_kubeflow_amd/apiserver/store.py (the in-process Python store)
// and the behaviour the reference's envtest suites rely on
// (kf/controllers/suite_test.go:50-104, odh/controllers/suite_test.go:91-275):
//
//   * resourceVersion (global counter), uid, creationTimestamp, generation,
//     generateName, optimistic concurrency (409 Conflict on a stale resourceVersion);
//   * status subresource isolation; finalizers + deletionTimestamp; no-op writes do
//     not bump the resourceVersion;
//   * merge, JSON and strategic-merge (list-by-merge-key subset) patches;
//   * label / field selectors for list and watch; watch resumption from a
//     resourceVersion with a bounded per-resource history (410 Expired when too old);
//   * mutating admission webhooks from MutatingWebhookConfiguration objects over
//     HTTPS (OpenSSL, caBundle verification, failurePolicy, Service → Endpoints
//     resolution round-robin over replicas), admission runs outside the store lock;
//   * ownerReference garbage collection (background + foreground) when --gc is set;
//   * kube-apiserver defaulting of Pods / StatefulSets / Deployments / Services on every write
//     (api_defaults; the same rules as models/defaults.py), config key "defaulting";
//   * discovery documents; bearer-token authentication.
//
// Concurrency: one thread per client connection (keep-alive); a store lock PER RESOURCE
// held only for commits (updates are prepared and compared outside it) — writes of
// different kinds never wait for each other, as in kube-apiserver, whose storage has no
// global lock — with the resourceVersion counter an atomic taken under the resource's lock
// (so each resource's events are in resourceVersion order), and the garbage collector's
// owner / uid indexes under a short lock of their own; cross-resource work (GC cascades,
// foreground-deletion owners) runs after the commit, each object under its own resource's
// lock.  A per-resource history lock the watch threads wait, wake and scan under (a watcher
// is woken only for events its namespace / selector admits); every stored object is an
// immutable shared snapshot, so readers and watchers never copy under a lock and each watch
// event is serialised once.  The watch history is bounded per resource (--history events;
// a namespace's history is the subsequence of its resource's, trimmed with it and dropped
// once empty and unwatched), so memory does not grow with the number of namespaces.
//
// --write-latency-ms D adds D ms to every write before it commits (outside any lock): an
// etcd-like storage round trip, for measurements that should not assume a free store.
//
// Usage: odh-apiserver --config scheme.json [--host 127.0.0.1] [--port 0] [--gc]
//        [--token T] [--history 512] [--write-latency-ms 0] [--webhook-connections 16];
//        prints "LISTENING <port>" once ready.

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <signal.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <malloc.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <ctime>
#include <deque>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <regex>
#include <set>
#include <sstream>
#include <thread>
#include <tuple>
#include <unordered_map>

#include "json.hpp"

using kj::T;
using kj::Value;

namespace {

// ------------------------------------------------------------------ errors

struct ApiErr {
  int code;
  std::string reason;
  std::string message;
  Value details;
};

Value status_obj(const ApiErr& e) {
  Value s = Value::object();
  s["kind"] = Value::str("Status");
  s["apiVersion"] = Value::str("v1");
  s["metadata"] = Value::object();
  s["status"] = Value::str("Failure");
  s["message"] = Value::str(e.message);
  s["reason"] = Value::str(e.reason);
  s["details"] = e.details.is_null() ? Value::object() : e.details;
  s["code"] = Value::integer(e.code);
  return s;
}

Value name_details(const std::string& name, const std::string& kind) {
  Value d = Value::object();
  d["name"] = Value::str(name);
  d["kind"] = Value::str(kind);
  return d;
}
ApiErr NotFound(const std::string& res, const std::string& name) {
  return {404, "NotFound", res + " \"" + name + "\" not found", name_details(name, res)};
}
ApiErr AlreadyExists(const std::string& res, const std::string& name) {
  return {409, "AlreadyExists", res + " \"" + name + "\" already exists", name_details(name, res)};
}
ApiErr Conflict(const std::string& res, const std::string& name, const std::string& msg = "") {
  return {409, "Conflict",
          "Operation cannot be fulfilled on " + res + " \"" + name + "\": " +
              (msg.empty() ? "the object has been modified; please apply your changes to the latest version and try "
                             "again"
                           : msg),
          name_details(name, res)};
}
ApiErr Invalid(const std::string& res, const std::string& name, const std::string& msg) {
  return {422, "Invalid", res + " \"" + name + "\" is invalid: " + msg, name_details(name, res)};
}
ApiErr BadRequest(const std::string& msg) { return {400, "BadRequest", msg, Value()}; }
ApiErr Forbidden(const std::string& msg) { return {403, "Forbidden", msg, Value()}; }
ApiErr NoKindMatch(const std::string& kind) {
  return {404, "NoKindMatch", "no matches for kind \"" + kind + "\" in version", Value()};
}
ApiErr Gone() { return {410, "Expired", "too old resource version", Value()}; }
ApiErr Internal(const std::string& msg) { return {500, "InternalError", msg, Value()}; }

// ------------------------------------------------------------------ scheme

struct Res {
  std::string group, kind, plural, singular, list_kind, storage, key;
  std::vector<std::string> versions, short_names;
  bool namespaced = true, status = false, installed = true;
  std::string err_res() const { return group.empty() ? plural : plural + "." + group; }
  std::string api_version(const std::string& v) const { return group.empty() ? v : group + "/" + v; }
};

std::vector<std::unique_ptr<Res>> g_res;
Res* by_plural(const std::string& g, const std::string& p) {
  for (auto& r : g_res)
    if (r->group == g && r->plural == p) return r.get();
  return nullptr;
}
Res* by_kind(const std::string& g, const std::string& k) {
  for (auto& r : g_res)
    if (r->group == g && r->kind == k) return r.get();
  return nullptr;
}
Res* by_key(const std::string& key) {
  for (auto& r : g_res)
    if (r->key == key) return r.get();
  return nullptr;
}

// ------------------------------------------------------------------ small utils

std::string rfc3339_now() {
  time_t t = time(nullptr);
  struct tm tm;
  gmtime_r(&t, &tm);
  char buf[32];
  strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

thread_local std::mt19937_64 t_rng{std::random_device{}() ^ (uint64_t)std::hash<std::thread::id>()(std::this_thread::get_id())};

std::string uuid4() {
  uint64_t a = t_rng(), b = t_rng();
  a = (a & 0xFFFFFFFFFFFF0FFFULL) | 0x0000000000004000ULL;
  b = (b & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;
  char buf[40];
  snprintf(buf, sizeof(buf), "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xFFFF),
           (unsigned)(a & 0xFFFF), (unsigned)(b >> 48), (unsigned long long)(b & 0xFFFFFFFFFFFFULL));
  return buf;
}

std::string rand_suffix(int n = 5) {
  static const char* al = "bcdfghjklmnpqrstvwxz2456789";
  std::string s;
  for (int k = 0; k < n; ++k) s += al[t_rng() % 27];
  return s;
}

const Value* md(const Value& o) { return o.get("metadata"); }
std::string mget(const Value& o, const char* k) {
  const Value* m = md(o);
  return m ? m->str_or(k) : "";
}
Value& mdm(Value& o) {
  Value& m = o["metadata"];
  if (!m.is_obj()) m = Value::object();
  return m;
}

std::string url_decode(const std::string& s) {
  std::string o;
  for (size_t n = 0; n < s.size(); ++n) {
    if (s[n] == '%' && n + 2 < s.size() && std::isxdigit((unsigned char)s[n + 1]) &&
        std::isxdigit((unsigned char)s[n + 2])) {
      o += (char)std::stoi(s.substr(n + 1, 2), nullptr, 16);
      n += 2;
    } else if (s[n] == '+') {
      o += ' ';
    } else {
      o += s[n];
    }
  }
  return o;
}

std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == d) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

// ------------------------------------------------------------------ selectors

struct LReq {
  std::string key, op;
  std::vector<std::string> vals;
};

std::vector<LReq> parse_labels(const std::string& text) {
  std::vector<LReq> out;
  std::vector<std::string> parts;
  std::string cur;
  int depth = 0;
  for (char c : text) {
    if (c == '(') depth++;
    if (c == ')') depth--;
    if (c == ',' && depth == 0) {
      parts.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  parts.push_back(cur);
  for (auto p : parts) {
    p = trim(p);
    if (p.empty()) continue;
    size_t sp = p.find(' ');
    if (sp != std::string::npos && p.find('(') != std::string::npos) {
      std::string k = trim(p.substr(0, sp));
      std::string rest = trim(p.substr(sp));
      std::string op = rest.rfind("notin", 0) == 0 ? "notin" : "in";
      size_t a = rest.find('('), b = rest.rfind(')');
      LReq r{k, op, {}};
      for (auto& v : split(rest.substr(a + 1, b - a - 1), ','))
        if (!trim(v).empty()) r.vals.push_back(trim(v));
      out.push_back(r);
      continue;
    }
    if (p[0] == '!') {
      out.push_back({trim(p.substr(1)), "!", {}});
      continue;
    }
    size_t e;
    if ((e = p.find("==")) != std::string::npos) out.push_back({trim(p.substr(0, e)), "=", {trim(p.substr(e + 2))}});
    else if ((e = p.find("!=")) != std::string::npos)
      out.push_back({trim(p.substr(0, e)), "!=", {trim(p.substr(e + 2))}});
    else if ((e = p.find('=')) != std::string::npos)
      out.push_back({trim(p.substr(0, e)), "=", {trim(p.substr(e + 1))}});
    else out.push_back({p, "exists", {}});
  }
  return out;
}

bool match_labels(const std::vector<LReq>& reqs, const Value& obj) {
  const Value* m = md(obj);
  const Value* labels = m ? m->get("labels") : nullptr;
  for (auto& r : reqs) {
    const Value* v = labels ? labels->get(r.key) : nullptr;
    bool has = v && v->is_str();
    std::string s = has ? v->s : "";
    if (r.op == "=") {
      if (!has || s != r.vals[0]) return false;
    } else if (r.op == "!=") {
      if (has && s == r.vals[0]) return false;
    } else if (r.op == "in") {
      if (!has || std::find(r.vals.begin(), r.vals.end(), s) == r.vals.end()) return false;
    } else if (r.op == "notin") {
      if (has && std::find(r.vals.begin(), r.vals.end(), s) != r.vals.end()) return false;
    } else if (r.op == "exists") {
      if (!has) return false;
    } else if (r.op == "!") {
      if (has) return false;
    }
  }
  return true;
}

struct FReq {
  std::vector<std::string> path;
  bool eq;
  std::string val;
};

std::vector<FReq> parse_fields(const std::string& text) {
  std::vector<FReq> out;
  for (auto p : split(text, ',')) {
    p = trim(p);
    if (p.empty()) continue;
    size_t e;
    if ((e = p.find("!=")) != std::string::npos) out.push_back({split(trim(p.substr(0, e)), '.'), false, trim(p.substr(e + 2))});
    else if ((e = p.find("==")) != std::string::npos)
      out.push_back({split(trim(p.substr(0, e)), '.'), true, trim(p.substr(e + 2))});
    else if ((e = p.find('=')) != std::string::npos)
      out.push_back({split(trim(p.substr(0, e)), '.'), true, trim(p.substr(e + 1))});
  }
  return out;
}

std::string scalar_str(const Value* v) {
  if (!v || v->is_null()) return "";
  if (v->t == T::String) return v->s;
  if (v->t == T::Bool) return v->b ? "True" : "False";
  return kj::dump(*v);
}

bool match_fields(const std::vector<FReq>& reqs, const Value& obj) {
  for (auto& r : reqs) {
    const Value* cur = &obj;
    for (auto& k : r.path) {
      cur = cur && cur->is_obj() ? cur->get(k) : nullptr;
    }
    if ((scalar_str(cur) == r.val) != r.eq) return false;
  }
  return true;
}

// ------------------------------------------------------------------ patches

struct PatchErr {
  std::string msg;
};

std::string unescape_tok(std::string t) {
  size_t p;
  while ((p = t.find("~1")) != std::string::npos) t.replace(p, 2, "/");
  while ((p = t.find("~0")) != std::string::npos) t.replace(p, 2, "~");
  return t;
}

std::vector<std::string> ptr_tokens(const std::string& path) {
  if (path.empty()) return {};
  if (path[0] != '/') throw PatchErr{"invalid JSON pointer " + path};
  std::vector<std::string> out;
  for (auto& t : split(path.substr(1), '/')) out.push_back(unescape_tok(t));
  return out;
}

// RFC 6901 array index: "0" or a digit string without a leading zero (no sign, blanks or
// trailing junk — std::stoul would take "1x", " 1" and "+1", and throw on "x")
size_t ptr_index(const std::string& t) {
  bool ok = !t.empty() && t.size() <= 9 && (t == "0" || t[0] != '0');
  for (char ch : t) ok = ok && ch >= '0' && ch <= '9';
  if (!ok) throw PatchErr{"bad list index " + t};
  return (size_t)std::stoul(t);
}

Value* ptr_get(Value& doc, const std::vector<std::string>& toks, size_t upto) {
  Value* cur = &doc;
  for (size_t n = 0; n < upto; ++n) {
    const std::string& t = toks[n];
    if (cur->is_obj()) {
      cur = cur->get(t);
      if (!cur) throw PatchErr{"path segment '" + t + "' not found"};
    } else if (cur->is_arr()) {
      size_t idx = ptr_index(t);
      if (idx >= cur->arr.size()) throw PatchErr{"bad list index " + t};
      cur = &cur->arr[idx];
    } else {
      throw PatchErr{"cannot traverse into scalar"};
    }
  }
  return cur;
}

void ptr_add(Value& doc, const std::vector<std::string>& toks, Value v) {
  if (toks.empty()) {
    doc = std::move(v);
    return;
  }
  Value* parent = ptr_get(doc, toks, toks.size() - 1);
  const std::string& last = toks.back();
  if (parent->is_obj()) {
    (*parent)[last] = std::move(v);
  } else if (parent->is_arr()) {
    if (last == "-") {
      parent->arr.push_back(std::move(v));
    } else {
      size_t idx = ptr_index(last);
      if (idx > parent->arr.size()) throw PatchErr{"list index out of range"};
      parent->arr.insert(parent->arr.begin() + idx, std::move(v));
    }
  } else {
    throw PatchErr{"cannot add into scalar"};
  }
}

Value ptr_remove(Value& doc, const std::vector<std::string>& toks) {
  if (toks.empty()) throw PatchErr{"cannot remove document root"};
  Value* parent = ptr_get(doc, toks, toks.size() - 1);
  const std::string& last = toks.back();
  if (parent->is_obj()) {
    Value* v = parent->get(last);
    if (!v) throw PatchErr{"remove: '" + last + "' not found"};
    Value out = std::move(*v);
    parent->erase(last);
    return out;
  }
  if (parent->is_arr()) {
    size_t idx = ptr_index(last);
    if (idx >= parent->arr.size()) throw PatchErr{"remove: bad index"};
    Value out = std::move(parent->arr[idx]);
    parent->arr.erase(parent->arr.begin() + idx);
    return out;
  }
  throw PatchErr{"cannot remove from scalar"};
}

Value apply_json_patch(Value doc, const Value& ops) {
  if (!ops.is_arr()) throw PatchErr{"JSON patch must be an array"};
  for (auto& op : ops.arr) {
    std::string kind = op.str_or("op");
    auto toks = ptr_tokens(op.str_or("path"));
    const Value* val = op.get("value");
    if (kind == "add") {
      ptr_add(doc, toks, val ? *val : Value());
    } else if (kind == "remove") {
      ptr_remove(doc, toks);
    } else if (kind == "replace") {
      if (toks.empty()) {
        doc = val ? *val : Value();
        continue;
      }
      Value* tgt = ptr_get(doc, toks, toks.size());
      *tgt = val ? *val : Value();
    } else if (kind == "move") {
      Value v = ptr_remove(doc, ptr_tokens(op.str_or("from")));
      ptr_add(doc, toks, std::move(v));
    } else if (kind == "copy") {
      auto ft = ptr_tokens(op.str_or("from"));
      Value v = *ptr_get(doc, ft, ft.size());
      ptr_add(doc, toks, std::move(v));
    } else if (kind == "test") {
      if (!(*ptr_get(doc, toks, toks.size()) == (val ? *val : Value())))
        throw PatchErr{"test failed at " + op.str_or("path")};
    } else {
      throw PatchErr{"unknown op " + kind};
    }
  }
  return doc;
}

Value merge_patch(const Value& target, const Value& patch) {
  if (!patch.is_obj()) return patch;
  Value out = target.is_obj() ? target : Value::object();
  for (auto& m : patch.obj) {
    if (m.v.is_null()) out.erase(m.k);
    else if (m.v.is_obj()) {
      const Value* cur = out.get(m.k);
      out[m.k] = merge_patch(cur ? *cur : Value(), m.v);
    } else {
      out[m.k] = m.v;
    }
  }
  return out;
}

const char* smp_key(const std::string& field, bool* known) {
  static const std::pair<const char*, const char*> keys[] = {
      {"containers", "name"}, {"initContainers", "name"}, {"ephemeralContainers", "name"}, {"env", "name"},
      {"volumes", "name"},    {"volumeMounts", "mountPath"}, {"ports", "containerPort"}, {"imagePullSecrets", "name"},
      {"tolerations", nullptr}, {"finalizers", nullptr}, {"ownerReferences", "uid"}, {"conditions", "type"}};
  for (auto& kv : keys)
    if (field == kv.first) {
      *known = true;
      return kv.second;
    }
  *known = false;
  return nullptr;
}

Value strategic_patch(const Value& target, const Value& patch) {
  if (!patch.is_obj()) return patch;
  Value out = target.is_obj() ? target : Value::object();
  for (auto& m : patch.obj) {
    if (!m.k.empty() && m.k[0] == '$') continue;
    bool known;
    const char* key = smp_key(m.k, &known);
    const Value* cur = out.get(m.k);
    if (m.v.is_null()) {
      out.erase(m.k);
    } else if (m.v.is_obj()) {
      out[m.k] = strategic_patch(cur ? *cur : Value(), m.v);
    } else if (m.v.is_arr() && key && cur && cur->is_arr()) {
      Value merged = *cur;
      for (auto& item : m.v.arr) {
        const Value* kv = item.is_obj() ? item.get(key) : nullptr;
        if (!kv) {
          merged.arr.push_back(item);
          continue;
        }
        int idx = -1;
        for (size_t n = 0; n < merged.arr.size(); ++n) {
          const Value* ek = merged.arr[n].is_obj() ? merged.arr[n].get(key) : nullptr;
          if (ek && *ek == *kv) {
            idx = (int)n;
            break;
          }
        }
        if (item.str_or("$patch") == "delete") {
          if (idx >= 0) merged.arr.erase(merged.arr.begin() + idx);
          continue;
        }
        if (idx < 0) merged.arr.push_back(item);
        else merged.arr[idx] = strategic_patch(merged.arr[idx], item);
      }
      out[m.k] = std::move(merged);
    } else {
      out[m.k] = m.v;
    }
  }
  return out;
}

// ------------------------------------------------------------------ store

using Obj = std::shared_ptr<const Value>;

struct EvCache {
  std::mutex mu;
  std::string version;
  std::shared_ptr<std::string> line;
};

struct Ev {
  int64_t seq;
  int64_t rv;
  const char* type;
  Obj obj;
  Obj old;
  std::shared_ptr<EvCache> cache;
  uint64_t t_ns = 0;  // committed at (mono_ns): the stall watchdog's watch-delivery delay
};

struct Hist;

struct WatchSlot {
  std::condition_variable cv;
  // the watch's namespace / label / field filter: emit() wakes a watcher only for events it
  // will deliver, so e.g. one node agent's label-selected cluster-wide pod watch is not
  // woken by every other GPU's pod writes
  std::function<bool(const Value&)> wants;
  // a label / field selector: events in the watch's history may be ones it never wants, so it
  // is not woken by them and could fall behind the bounded history — the periodic wake-up
  // (emit) advances it; a watch without one is woken by every event it reads
  bool filtered = false;
  // the history it reads and the seq it has scanned up to (both under the bucket's hmu): the
  // periodic wake-up skips a watcher with nothing unscanned
  const Hist* hist = nullptr;
  int64_t seen = 0;
};

// one ordered event history: `seq` numbers its events, `hist` keeps the newest S.history
struct Hist {
  std::deque<Ev> hist;
  int64_t seq = 0;
};

struct Bucket {
  std::map<std::pair<std::string, std::string>, Obj> objs;
  // every event of the kind (cluster-wide watchers) and, per namespace, that namespace's
  // events: a namespace-scoped watch scans only its own namespace's history, so with one
  // control-plane shard per GPU rank a woken watcher reads its events, not every rank's
  // (the scan was O(ranks) per event).  Element references of by_ns stay valid (node-based).
  Hist all;
  std::unordered_map<std::string, Hist> by_ns;
  // watchers by namespace ("" = cluster-wide): a write wakes only the watchers of its kind
  // AND namespace, so with one control-plane shard per GPU rank (each watching its own
  // namespaces) a write costs O(1) wake-ups instead of one per shard
  std::unordered_multimap<std::string, std::shared_ptr<WatchSlot>> watchers;
  // rv of the newest event trimmed off `all` (0: none yet): a watch resuming from an older
  // resourceVersion may have missed events and gets 410 Gone
  int64_t dropped_rv = 0;
  // hist / seq / watchers have their own lock: watch streams wait, wake and scan under it
  // without touching the store lock the request threads commit under (lock order: the
  // resource's store lock, then this one — emit() runs inside a commit)
  std::mutex hmu;
  // this resource's store lock: objs, and the commit order of its events
  std::mutex mu;
  std::atomic<uint64_t> wait_ns{0}, contended{0};  // contended acquisitions of mu (GET /metrics "locks")
};

struct Store {
  std::unordered_map<std::string, Bucket> data;  // one per resource, created at start-up, never rehashed
  std::atomic<int64_t> rv{0};
  // 512 events per resource: at 4 ranks x 300 steps on the MI355X box, 155 vs 210 MiB resident
  // for the same notebooks/s and no watch answered 410 Gone, nor in 64-notebook bursts or the
  // 8-rank CPU rehearsal (profiles/r4_hist)
  size_t history = 512;
  std::atomic<int64_t> write_latency_us{0};  // --write-latency-ms; POST /debug/storage-latency
  bool gc = false;
  bool defaulting = true;  // kube-apiserver defaulting of Pods / StatefulSets / Deployments / Services
  std::atomic<uint64_t> requests{0}, writes{0}, webhook_calls{0};
} S;

// The garbage collector's indexes — owner uid → dependents, uid → object — striped by uid:
// every access is about one uid, so writers of different objects (every rank's commits, in
// every resource) do not meet on one mutex.  A stripe's lock is taken inside a resource's
// store lock, never around one, and never two stripes at once.
using ObjKey = std::tuple<std::string, std::string, std::string>;
struct IdxStripe {
  std::mutex mu;
  std::unordered_map<std::string, std::set<ObjKey>> owners;
  std::unordered_map<std::string, ObjKey> uids;
};
constexpr size_t kIdxStripes = 64;
IdxStripe g_idx[kIdxStripes];
IdxStripe& idx(const std::string& uid) { return g_idx[std::hash<std::string>{}(uid) & (kIdxStripes - 1)]; }

// Where the server's CPU goes (GET /metrics "prof"): thread CPU time per request class,
// store-lock contention on the request path, watch wake-ups and the history entries the
// woken watchers scanned, wall time spent waiting on admission webhooks.
enum Cat { C_GET, C_LIST, C_CREATE, C_UPDATE, C_PATCH, C_DELETE, C_WATCH, C_OTHER, C_N };
const char* const CAT_NAMES[C_N] = {"get", "list", "create", "update", "patch", "delete", "watch", "other"};
struct Prof {
  std::atomic<uint64_t> cpu_ns[C_N]{}, calls[C_N]{};
  std::atomic<uint64_t> lock_wait_ns{0}, lock_contended{0}, wakeups{0}, scanned{0}, admit_wall_ns{0};
  std::atomic<uint64_t> lock_hold_ns[C_N]{};
  std::atomic<uint64_t> trim_ns{0}, trim_max_ns{0}, trims{0};  // malloc_trim passes (allocations wait on them)
  std::atomic<uint64_t> webhook_dials{0}, webhook_dial_ns{0};  // new webhook connections: connect + TLS handshake
  std::atomic<uint64_t> watch_gone{0};  // watches answered 410 Gone (behind the bounded history): each is a relist
} P;
thread_local int t_cat = C_OTHER;

// thread CPU per phase of the write path (GET /metrics "phases"): where a write's CPU goes
enum Phase { PH_PARSE, PH_ADMIT, PH_VALIDATE, PH_DEFAULTS, PH_PATCH, PH_PREPARE, PH_DUMP, PH_N };
const char* const PHASE_NAMES[PH_N] = {"parse", "admit", "validate", "defaults", "patch", "prepare", "dump"};
std::atomic<uint64_t> g_phase_ns[PH_N]{};
uint64_t thread_cpu_ns();
struct PhaseTimer {
  int ph;
  uint64_t t0;
  explicit PhaseTimer(int p) : ph(p), t0(thread_cpu_ns()) {}
  ~PhaseTimer() { g_phase_ns[ph] += thread_cpu_ns() - t0; }
};

// every admission webhook call's wall time in µs, the newest 65536 (GET /debug/admissions?from=N
// answers those from call N on): admission latency percentiles under a burst of creates
constexpr uint64_t kAdmitRing = 1 << 16;
struct AdmitRing {
  std::atomic<uint64_t> seq{0};
  std::atomic<uint32_t> us[kAdmitRing];
} g_admit;

uint64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// the whole process, exited connection threads included (the benchmark's CPU accounting)
uint64_t process_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// ODH_STALL_WATCHDOG_MS (diagnostics, main()): stalls at least this long are reported to stderr
int g_stall_ms = 0;

uint64_t mono_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the store lock on the request path, timing only the contended acquisitions
// Watcher wake-ups are decided and delivered after the store lock is released: emit()
// (which runs inside a commit) only queues the candidate watchers of the event on this
// thread; ~StoreLock evaluates their filters and notifies them once the lock is free, so
// the lock covers the commit alone (with one shard per GPU a pod write has a candidate
// per node-agent watch).  No wake-up is lost: the event is published (seq bumped) under
// the history lock before the notify, and a waiter re-checks seq under that lock.
struct PendingWake {
  std::shared_ptr<WatchSlot> w;
  Obj obj, old;
  bool all;
};
thread_local std::vector<PendingWake> t_wake;
// events trimmed off a bounded history inside a commit: often the last reference to an old
// object version, whose tree is freed once the store lock is released (~StoreLock), not
// while every other writer of the resource waits for it
thread_local std::vector<Ev> t_free;
thread_local std::vector<std::shared_ptr<std::string>> t_free_lines;
// an event's serialised watch line is dropped this many events after it was emitted: every
// live watcher has written it by then (they are woken at once); a late reader re-serialises.
// The history keeps the objects (shared with the store) but not a second, JSON copy of each
constexpr size_t kLineKeep = 64;
// Owners removed by this thread whose dependents the garbage collector has yet to delete:
// the cascade runs after the removing commit has released the store lock (each owner's
// dependents under a lock of their own, still before the request is answered), so a
// finalizer-removal update or a delete holds the lock for its own object only.
thread_local std::vector<std::string> t_gc;
thread_local bool t_gc_running = false;
void run_gc() noexcept;

void flush_wakes() {
  std::vector<PendingWake> ws;
  ws.swap(t_wake);
  for (auto& p : ws) {
    WatchSlot* w = p.w.get();
    if (p.all || !w->wants || w->wants(*p.obj) || (p.old && w->wants(*p.old))) w->cv.notify_all();
  }
}

// Commits hold the lock for a few microseconds, less than a futex sleep + wake-up costs the
// waiter: a contended acquisition spins briefly before it parks, as Go's sync.Mutex (the
// kube-apiserver's) does — 4 rounds of 30 PAUSEs, then it sleeps.
constexpr int kSpinRounds = 4, kSpinPauses = 30;

// owners whose foreground-deletion finalizer may be due (a dependent of theirs was removed):
// re-checked after the commit, under the owner's resource lock (fg_recheck)
thread_local std::vector<std::string> t_fg;

// one resource's store lock on the request path, timing only the contended acquisitions
struct StoreLock {
  std::mutex& mu;
  Bucket& b;
  uint64_t t_acq;
  explicit StoreLock(Bucket& b);
  ~StoreLock() {
    P.lock_hold_ns[t_cat] += mono_ns() - t_acq;  // who keeps the others waiting
    mu.unlock();
    if (!t_free.empty()) t_free.clear();
    if (!t_free_lines.empty()) t_free_lines.clear();
    if (!t_wake.empty()) flush_wakes();
    if ((!t_gc.empty() || !t_fg.empty()) && !t_gc_running) run_gc();
  }
  StoreLock(const StoreLock&) = delete;
  StoreLock& operator=(const StoreLock&) = delete;
};

StoreLock::StoreLock(Bucket& bk) : mu(bk.mu), b(bk) {
  if (!mu.try_lock()) {
    uint64_t t0 = mono_ns();
    bool got = false;
    for (int r = 0; r < kSpinRounds && !got; ++r) {
      for (int i = 0; i < kSpinPauses; ++i) __builtin_ia32_pause();
      got = mu.try_lock();
    }
    if (!got) mu.lock();
    uint64_t w = mono_ns() - t0;
    P.lock_wait_ns += w;
    P.lock_contended++;
    b.wait_ns += w;
    b.contended++;
  }
  t_acq = mono_ns();
}

// S.data holds every resource from start-up on (init_buckets) and never changes shape, so
// looking a bucket up needs no lock
Bucket& bucket(const Res& r) { return S.data.find(r.key)->second; }

void init_buckets() {
  S.data.reserve(g_res.size() * 2);
  for (auto& r : g_res) S.data[r->key];
}

// an etcd-like storage round trip before a write commits (--write-latency-ms), no lock held
void storage_latency() {
  const int64_t us = S.write_latency_us.load(std::memory_order_relaxed);
  if (us > 0) std::this_thread::sleep_for(std::chrono::microseconds(us));
}

void index_owner(const Res& r, const Value& o, bool remove) {
  const Value* m = md(o);
  const Value* refs = m ? m->get("ownerReferences") : nullptr;
  if (!refs || !refs->is_arr()) return;
  auto k = std::make_tuple(r.key, mget(o, "namespace"), mget(o, "name"));
  for (auto& ref : refs->arr) {
    std::string u = ref.str_or("uid");
    if (u.empty()) continue;
    IdxStripe& st = idx(u);
    std::lock_guard<std::mutex> ig(st.mu);
    if (remove) {
      auto it = st.owners.find(u);
      if (it != st.owners.end()) {
        it->second.erase(k);
        if (it->second.empty()) st.owners.erase(it);
      }
    } else {
      st.owners[u].insert(k);
    }
  }
}

// callers hold the resource's store lock
void emit(const Res& r, const char* type, Obj obj, Obj old) {
  Bucket& b = bucket(r);
  std::lock_guard<std::mutex> hg(b.hmu);
  const std::string evns = mget(*obj, "namespace");
  Ev e{++b.all.seq, std::stoll(mget(*obj, "resourceVersion")), type, std::move(obj), std::move(old),
       std::make_shared<EvCache>()};
  if (!evns.empty()) {
    Hist& h = b.by_ns[evns];
    Ev copy = e;  // the same event (shared object, old object and serialisation cache)
    copy.seq = ++h.seq;
    h.hist.push_back(std::move(copy));
  }
  b.all.hist.push_back(std::move(e));
  while (b.all.hist.size() > S.history) {
    // a namespace's history is the subsequence of the resource's: trim both together, so the
    // history holds at most --history events per resource however many namespaces there are
    const Ev& old = b.all.hist.front();
    b.dropped_rv = old.rv;
    const std::string ons = mget(*old.obj, "namespace");
    if (!ons.empty()) {
      auto it = b.by_ns.find(ons);
      if (it != b.by_ns.end() && !it->second.hist.empty() && it->second.hist.front().rv == old.rv) {
        t_free.push_back(std::move(it->second.hist.front()));
        it->second.hist.pop_front();
        // an idle, unwatched namespace (e.g. deleted) keeps nothing; a watcher's Hist& stays valid
        if (it->second.hist.empty() && ons != evns && !b.watchers.count(ons)) b.by_ns.erase(it);
      }
    }
    t_free.push_back(std::move(b.all.hist.front()));
    b.all.hist.pop_front();
  }
  if (b.all.hist.size() > kLineKeep) {
    EvCache& c = *b.all.hist[b.all.hist.size() - 1 - kLineKeep].cache;
    std::unique_lock<std::mutex> cl(c.mu, std::try_to_lock);  // a watcher serialising it: next time
    if (cl.owns_lock() && c.line) t_free_lines.push_back(std::move(c.line));
  }
  if (g_stall_ms > 0) {
    const uint64_t now = mono_ns();
    b.all.hist.back().t_ns = now;
    if (!evns.empty()) b.by_ns[evns].hist.back().t_ns = now;
  }
  const Ev& ev = b.all.hist.back();
  const int64_t step = std::max<int64_t>(1, (int64_t)S.history / 16);
  if (b.all.seq % step == 0) {
    // periodic wake-up of the selector-filtered watchers, an eighth of them every history/16
    // events (each one every half history): one that rejects every event it sees advances
    // past them before they fall off the bounded history (no spurious 410 Gone relists),
    // without waking every watcher of the resource at once (a herd on the history lock that
    // commits then wait for).  Only a watcher whose history moved since its last scan: with
    // one watch per namespace most of them (every idle namespace's) have nothing to skip
    const int64_t turn = (b.all.seq / step) & 7;
    int64_t i = 0;
    for (auto& w : b.watchers) {
      WatchSlot& s = *w.second;
      if (s.filtered && (i++ & 7) == turn && (!s.hist || s.hist->seq > s.seen))
        t_wake.push_back({w.second, ev.obj, ev.old, true});
    }
  }
  auto wake = [&](const std::string& ns) {
    auto rg = b.watchers.equal_range(ns);
    for (auto it = rg.first; it != rg.second; ++it) t_wake.push_back({it->second, ev.obj, ev.old, false});
  };
  const std::string ns = mget(*ev.obj, "namespace");
  wake(ns);
  if (!ns.empty()) wake("");
}

Value out_obj(const Res& r, const Value& o, const std::string& version) {
  Value c = o;
  if (!version.empty() && version != r.storage) c["apiVersion"] = Value::str(r.api_version(version));
  return c;
}

// a and b agree on every member not named in skip (object members in any order); no copies
bool members_equal_except(const Value& a, const Value& b, std::initializer_list<const char*> skip) {
  auto skipped = [&](const std::string& k) {
    for (const char* x : skip)
      if (k == x) return true;
    return false;
  };
  size_t na = 0, nb = 0;
  for (auto& m : a.obj) {
    if (skipped(m.k)) continue;
    ++na;
    const Value* o = b.get(m.k);
    if (!o || !(m.v == *o)) return false;
  }
  for (auto& m : b.obj)
    if (!skipped(m.k)) ++nb;
  return na == nb;
}

bool spec_equal(const Value& a, const Value& b) {
  // everything but metadata / status / apiVersion / kind
  return members_equal_except(a, b, {"metadata", "status", "apiVersion", "kind"});
}

bool equal_except_meta(const Value& a, const Value& b) {
  if (!members_equal_except(a, b, {"metadata"})) return false;
  const Value* ma = a.get("metadata");
  const Value* mb = b.get("metadata");
  if (!ma || !mb) return ma == mb;
  if (!ma->is_obj() || !mb->is_obj()) return *ma == *mb;
  return members_equal_except(*ma, *mb, {"resourceVersion", "managedFields", "generation"});
}

Value out_obj(const Res& r, const Value& o, const std::string& version);

// the response body of a write: no copy when the request used the storage version
std::string dump_out(const Res& r, const Value& o, const std::string& version) {
  PhaseTimer pt(PH_DUMP);
  if (version.empty() || version == r.storage) return kj::dump(o);
  return kj::dump(out_obj(r, o, version));
}

// ------------------------------------------------------------------ CRD structural schemas
// prune -> default -> validate on every write of a kind that has a schema (config key "schemas":
// plural.group -> openAPIV3Schema; the notebooks.kubeflow.org one is the reference's full PodSpec
// schema + validation_patches.yaml, generated by models/crd.py).  Same rules and error strings as
// models/openapi.py.

std::map<std::string, Value> g_schemas;

const char* type_name(const Value& v) {
  switch (v.t) {
    case T::Null: return "null";
    case T::Bool: return "boolean";
    case T::Int: return "integer";
    case T::Double: return "number";
    case T::String: return "string";
    case T::Array: return "array";
    default: return "object";
  }
}

std::string fmt_val(const Value& v) {
  switch (v.t) {
    case T::String: return "\"" + v.s + "\"";
    case T::Bool: return v.b ? "true" : "false";
    case T::Int: return std::to_string(v.i);
    case T::Double: {
      char b[64];
      snprintf(b, sizeof(b), "%g", v.d);
      return b;
    }
    case T::Null: return "null";
    default: return std::string("\"") + type_name(v) + "\"";
  }
}

bool schema_flag(const Value& s, const char* k) {
  const Value* v = s.get(k);
  return v && v->t == T::Bool && v->b;
}

bool type_ok(const Value& s, const Value& v) {
  if (schema_flag(s, "x-kubernetes-int-or-string")) return v.t == T::Int || v.t == T::String;
  std::string t = s.str_or("type");
  if (t.empty()) return true;
  if (t == "integer") return v.t == T::Int || (v.t == T::Double && v.d == (double)(int64_t)v.d);
  if (t == "number") return v.t == T::Int || v.t == T::Double;
  return t == type_name(v);
}

void schema_prune(const Value& s, Value& v, bool root) {
  if (v.is_obj()) {
    if (schema_flag(s, "x-kubernetes-preserve-unknown-fields")) return;
    const Value* props = s.get("properties");
    const Value* addl = s.get("additionalProperties");
    bool addl_true = addl && addl->t == T::Bool && addl->b;
    for (size_t n = 0; n < v.obj.size();) {
      kj::Member& m = v.obj[n];
      if (root && (m.k == "apiVersion" || m.k == "kind" || m.k == "metadata")) {
        ++n;
        continue;
      }
      const Value* sub = props ? props->get(m.k) : nullptr;
      if (!sub && addl && addl->is_obj()) sub = addl;
      if (!sub) {
        if (!addl_true) {
          v.obj.erase(v.obj.begin() + n);
          continue;
        }
        ++n;
        continue;
      }
      if (m.v.is_null() && !schema_flag(*sub, "nullable")) {
        v.obj.erase(v.obj.begin() + n);
        continue;
      }
      schema_prune(*sub, m.v, false);
      ++n;
    }
  } else if (v.is_arr()) {
    if (const Value* item = s.get("items"); item && item->is_obj())
      for (auto& x : v.arr) schema_prune(*item, x, false);
  }
}

void schema_default(const Value& s, Value& v) {
  if (v.is_obj()) {
    if (const Value* props = s.get("properties"); props && props->is_obj())
      for (auto& p : props->obj) {
        if (!v.get(p.k))
          if (const Value* d = p.v.get("default")) v[p.k] = *d;
        if (Value* x = v.get(p.k)) schema_default(p.v, *x);
      }
    if (const Value* addl = s.get("additionalProperties"); addl && addl->is_obj())
      for (auto& m : v.obj) schema_default(*addl, m.v);
  } else if (v.is_arr()) {
    if (const Value* item = s.get("items"); item && item->is_obj())
      for (auto& x : v.arr) schema_default(*item, x);
  }
}

const std::regex& cached_regex(const std::string& pat) {
  static std::mutex mu;
  static std::map<std::string, std::unique_ptr<std::regex>> cache;
  std::lock_guard<std::mutex> g(mu);
  auto& slot = cache[pat];
  if (!slot) slot = std::make_unique<std::regex>(pat, std::regex::ECMAScript | std::regex::optimize);
  return *slot;
}

void schema_validate(const Value& s, const Value& v, const std::string& path, std::vector<std::string>& errs) {
  if (!type_ok(s, v)) {
    std::string want = schema_flag(s, "x-kubernetes-int-or-string") ? "integer or string" : s.str_or("type");
    errs.push_back(path + ": Invalid value: " + fmt_val(v) + ": " + path + " in body must be of type " + want + ": \"" +
                   type_name(v) + "\"");
    return;
  }
  std::string fmt = s.str_or("format");
  if ((fmt == "int32") && v.t == T::Int && (v.i < INT32_MIN || v.i > INT32_MAX))
    errs.push_back(path + ": Invalid value: " + std::to_string(v.i) + ": " + path + " in body should be a valid int32");
  if (const Value* en = s.get("enum"); en && en->is_arr()) {
    bool ok = false;
    for (auto& x : en->arr) ok = ok || x == v;
    if (!ok) {
      std::string l;
      for (auto& x : en->arr) l += (l.empty() ? "" : ", ") + fmt_val(x);
      errs.push_back(path + ": Unsupported value: " + fmt_val(v) + ": supported values: " + l);
    }
  }
  if (const Value* pat = s.get("pattern"); pat && pat->is_str() && v.is_str())
    if (!std::regex_search(v.s, cached_regex(pat->s)))
      errs.push_back(path + ": Invalid value: " + fmt_val(v) + ": " + path + " in body should match '" + pat->s + "'");
  if (v.is_obj()) {
    const Value* props = s.get("properties");
    if (const Value* req = s.get("required"); req && req->is_arr())
      for (auto& r : req->arr)
        if (r.is_str() && !v.get(r.s)) errs.push_back((path.empty() ? "" : path + ".") + r.s + ": Required value");
    const Value* addl = s.get("additionalProperties");
    for (auto& m : v.obj) {
      const Value* sub = props ? props->get(m.k) : nullptr;
      if (!sub && addl && addl->is_obj()) sub = addl;
      if (sub && !(path.empty() && m.k == "metadata")) schema_validate(*sub, m.v, path.empty() ? m.k : path + "." + m.k, errs);
    }
  } else if (v.is_arr()) {
    if (const Value* mi = s.get("minItems"); mi && mi->t == T::Int && (int64_t)v.arr.size() < mi->i)
      errs.push_back(path + ": Invalid value: " + std::to_string(v.arr.size()) + ": " + path + " in body should have at least " +
                     std::to_string(mi->i) + " items");
    if (const Value* ma = s.get("maxItems"); ma && ma->t == T::Int && (int64_t)v.arr.size() > ma->i)
      errs.push_back(path + ": Too many: " + std::to_string(v.arr.size()) + ": must have at most " + std::to_string(ma->i) + " items");
    std::string lt = s.str_or("x-kubernetes-list-type");
    if (lt == "set") {
      for (size_t i = 0; i < v.arr.size(); ++i)
        for (size_t j = 0; j < i; ++j)
          if (v.arr[j] == v.arr[i]) {
            errs.push_back(path + "[" + std::to_string(i) + "]: Duplicate value: " + fmt_val(v.arr[i]));
            break;
          }
    } else if (lt == "map") {
      const Value* keys = s.get("x-kubernetes-list-map-keys");
      for (size_t i = 0; keys && keys->is_arr() && i < v.arr.size(); ++i)
        for (size_t j = 0; j < i; ++j) {
          bool same = v.arr[i].is_obj() && v.arr[j].is_obj();
          for (auto& k : keys->arr) {
            if (!same) break;
            const Value* a = v.arr[i].get(k.s);
            const Value* b = v.arr[j].get(k.s);
            same = (!a && !b) || (a && b && *a == *b);
          }
          if (same) {
            std::string d;
            for (auto& k : keys->arr) {
              const Value* a = v.arr[i].get(k.s);
              d += (d.empty() ? "" : ", ") + std::string("\"") + k.s + "\":" + (a ? fmt_val(*a) : "null");
            }
            errs.push_back(path + "[" + std::to_string(i) + "]: Duplicate value: {" + d + "}");
            break;
          }
        }
    }
    if (const Value* item = s.get("items"); item && item->is_obj())
      for (size_t i = 0; i < v.arr.size(); ++i) schema_validate(*item, v.arr[i], path + "[" + std::to_string(i) + "]", errs);
  }
}

std::optional<std::string> validate(const Res& r, Value& o) {
  PhaseTimer pt(PH_VALIDATE);
  auto it = g_schemas.find(r.key);
  if (it == g_schemas.end()) return std::nullopt;
  schema_prune(it->second, o, true);
  schema_default(it->second, o);
  std::vector<std::string> errs;
  schema_validate(it->second, o, "", errs);
  if (errs.empty()) return std::nullopt;
  if (errs.size() == 1) return errs[0];
  std::string all = "[";
  for (size_t n = 0; n < errs.size(); ++n) all += (n ? ", " : "") + errs[n];
  return all + "]";
}

// ------------------------------------------------------------------ kube-apiserver defaulting
// Same rules as models/defaults.py (k8s.io/kubernetes/pkg/apis/{core,apps}/v1/defaults.go plus
// resource.Quantity canonicalisation), applied to every Pod / StatefulSet / Deployment /
// Service write so controllers see the live objects a real apiserver would hand them.

void set_default(Value& o, const char* k, Value v) {
  if (!o.get(k)) o[k] = std::move(v);
}

Value& obj_at(Value& o, const char* k) {
  Value& v = o[k];
  if (!v.is_obj()) v = Value::object();
  return v;
}

// resource.Quantity -> canonical string ("0.5" -> "500m", "1024Mi" -> "1Gi", "1000" -> "1k");
// empty when the text is not a quantity (validation reports it elsewhere).
std::string canon_quantity(const std::string& text) {
  using i128 = __int128;
  size_t n = 0;
  bool neg = false;
  if (n < text.size() && (text[n] == '+' || text[n] == '-')) neg = text[n++] == '-';
  i128 num = 0, den = 1;
  bool digits = false, dot = false;
  for (; n < text.size(); ++n) {
    char c = text[n];
    if (c >= '0' && c <= '9') {
      if (num > ((i128)1 << 100)) return "";
      num = num * 10 + (c - '0');
      if (dot) den *= 10;
      digits = true;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!digits) return "";
  std::string suf = text.substr(n);
  bool binary = false;
  static const std::pair<const char*, int> bin[] = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  static const std::pair<const char*, int> dec[] = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                                    {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  int exp10 = 0;
  bool matched = false;
  for (auto& b : bin)
    if (suf == b.first) {
      num <<= b.second;
      binary = matched = true;
    }
  for (auto& d : dec)
    if (!matched && suf == d.first) {
      exp10 = d.second;
      matched = true;
    }
  if (!matched && (suf.size() >= 2 && (suf[0] == 'e' || suf[0] == 'E'))) {
    char* end = nullptr;
    long e = std::strtol(suf.c_str() + 1, &end, 10);
    if (*end || e > 18 || e < -18) return "";
    exp10 = (int)e;
    matched = true;
  }
  if (!matched) return "";
  for (; exp10 > 0; --exp10) num *= 10;
  for (; exp10 < 0; ++exp10) den *= 10;
  auto gcd = [](i128 a, i128 b) {
    while (b) {
      i128 t = a % b;
      a = b;
      b = t;
    }
    return a;
  };
  if (num == 0) return "0";
  i128 g = gcd(num, den);
  num /= g;
  den /= g;
  auto to_s = [](i128 v) {
    std::string out;
    if (v == 0) return std::string("0");
    while (v) {
      out.insert(out.begin(), char('0' + (int)(v % 10)));
      v /= 10;
    }
    return out;
  };
  std::string sign = neg ? "-" : "";
  if (binary) {
    for (int k = 5; k >= 0; --k) {
      i128 base = (i128)1 << bin[k].second;
      if (den == 1 && num % base == 0) return sign + to_s(num / base) + bin[k].first;
    }
    if (den == 1) return sign + to_s(num);
  }
  if (den == 1) {
    static const std::pair<const char*, int> up[] = {{"E", 18}, {"P", 15}, {"T", 12}, {"G", 9}, {"M", 6}, {"k", 3}};
    for (auto& u : up) {
      i128 p = 1;
      for (int k = 0; k < u.second; ++k) p *= 10;
      if (num % p == 0) return sign + to_s(num / p) + u.first;
    }
    return sign + to_s(num);
  }
  static const std::pair<const char*, int> down[] = {{"m", 3}, {"u", 6}, {"n", 9}};
  for (auto& d : down) {
    i128 p = 1;
    for (int k = 0; k < d.second; ++k) p *= 10;
    if ((num * p) % den == 0) return sign + to_s(num * p / den) + d.first;
  }
  i128 p = 1000000000;
  return sign + to_s(num * p / den) + "n";
}

void canon_quantities(Value* q) {
  if (!q || !q->is_obj()) return;
  for (auto& m : q->obj)
    if (m.v.is_str()) {
      std::string c = canon_quantity(m.v.s);
      if (!c.empty()) m.v.s = c;
    }
}

std::string image_pull_policy(const std::string& image) {
  if (image.find('@') != std::string::npos) return "IfNotPresent";
  std::string last = image.substr(image.rfind('/') == std::string::npos ? 0 : image.rfind('/') + 1);
  auto colon = last.rfind(':');
  std::string tag = colon == std::string::npos ? "" : last.substr(colon + 1);
  return tag.empty() || tag == "latest" ? "Always" : "IfNotPresent";
}

void default_probe(Value* p) {
  if (!p || !p->is_obj()) return;
  set_default(*p, "timeoutSeconds", Value::integer(1));
  set_default(*p, "periodSeconds", Value::integer(10));
  set_default(*p, "successThreshold", Value::integer(1));
  set_default(*p, "failureThreshold", Value::integer(3));
  if (Value* hg = p->get("httpGet"); hg && hg->is_obj()) {
    set_default(*hg, "path", Value::str("/"));
    set_default(*hg, "scheme", Value::str("HTTP"));
  }
}

void default_container(Value& c) {
  if (!c.is_obj()) return;
  set_default(c, "terminationMessagePath", Value::str("/dev/termination-log"));
  set_default(c, "terminationMessagePolicy", Value::str("File"));
  if (const Value* img = c.get("image"); img && img->is_str()) set_default(c, "imagePullPolicy", Value::str(image_pull_policy(img->s)));
  if (Value* ports = c.get("ports"); ports && ports->is_arr())
    for (auto& p : ports->arr)
      if (p.is_obj()) set_default(p, "protocol", Value::str("TCP"));
  if (Value* env = c.get("env"); env && env->is_arr())
    for (auto& e : env->arr) {
      Value* vf = e.get("valueFrom");
      Value* fr = vf ? vf->get("fieldRef") : nullptr;
      if (fr && fr->is_obj()) set_default(*fr, "apiVersion", Value::str("v1"));
    }
  Value& res = obj_at(c, "resources");
  canon_quantities(res.get("limits"));
  canon_quantities(res.get("requests"));
  for (const char* k : {"livenessProbe", "readinessProbe", "startupProbe"}) default_probe(c.get(k));
}

void default_pod_spec(Value& spec) {
  set_default(spec, "restartPolicy", Value::str("Always"));
  set_default(spec, "terminationGracePeriodSeconds", Value::integer(30));
  set_default(spec, "dnsPolicy", Value::str("ClusterFirst"));
  set_default(spec, "securityContext", Value::object());
  set_default(spec, "schedulerName", Value::str("default-scheduler"));
  set_default(spec, "enableServiceLinks", Value::boolean(true));
  if (!spec.str_or("serviceAccountName").empty() && spec.str_or("serviceAccount").empty())
    spec["serviceAccount"] = Value::str(spec.str_or("serviceAccountName"));
  for (const char* k : {"initContainers", "containers"})
    if (Value* cs = spec.get(k); cs && cs->is_arr())
      for (auto& c : cs->arr) default_container(c);
  if (Value* vols = spec.get("volumes"); vols && vols->is_arr())
    for (auto& v : vols->arr) {
      if (!v.is_obj()) continue;
      for (const char* src : {"secret", "configMap"})
        if (Value* x = v.get(src); x && x->is_obj()) set_default(*x, "defaultMode", Value::integer(420));
      if (Value* hp = v.get("hostPath"); hp && hp->is_obj()) set_default(*hp, "type", Value::str(""));
      if (Value* ed = v.get("emptyDir"); ed && ed->is_obj())
        if (Value* sl = ed->get("sizeLimit"); sl && sl->is_str()) {
          std::string c = canon_quantity(sl->s);
          if (!c.empty()) sl->s = c;
        }
    }
}

void default_template(Value& spec) {
  Value& t = obj_at(spec, "template");
  set_default(obj_at(t, "metadata"), "creationTimestamp", Value::null());
  default_pod_spec(obj_at(t, "spec"));
}

void api_defaults(const Res& r, Value& o) {
  PhaseTimer pt(PH_DEFAULTS);
  if (r.key == "statefulsets.apps" || r.key == "deployments.apps") {
    Value& spec = obj_at(o, "spec");
    if (const Value* rep = spec.get("replicas"); !rep || rep->is_null()) spec["replicas"] = Value::integer(1);
    set_default(spec, "revisionHistoryLimit", Value::integer(10));
    if (r.key == "statefulsets.apps") {
      set_default(spec, "podManagementPolicy", Value::str("OrderedReady"));
      Value& us = obj_at(spec, "updateStrategy");
      set_default(us, "type", Value::str("RollingUpdate"));
      if (us.str_or("type") == "RollingUpdate") set_default(obj_at(us, "rollingUpdate"), "partition", Value::integer(0));
      Value& ret = obj_at(spec, "persistentVolumeClaimRetentionPolicy");
      set_default(ret, "whenDeleted", Value::str("Retain"));
      set_default(ret, "whenScaled", Value::str("Retain"));
    } else {
      Value& st = obj_at(spec, "strategy");
      set_default(st, "type", Value::str("RollingUpdate"));
      if (st.str_or("type") == "RollingUpdate") {
        Value& ru = obj_at(st, "rollingUpdate");
        set_default(ru, "maxUnavailable", Value::str("25%"));
        set_default(ru, "maxSurge", Value::str("25%"));
      }
      set_default(spec, "progressDeadlineSeconds", Value::integer(600));
    }
    default_template(spec);
  } else if (r.key == "pods") {
    Value& spec = obj_at(o, "spec");
    for (const char* k : {"containers", "initContainers"})
      if (Value* cs = spec.get(k); cs && cs->is_arr())
        for (auto& c : cs->arr) {
          Value* res = c.get("resources");
          Value* lim = res ? res->get("limits") : nullptr;
          if (!lim || !lim->is_obj() || lim->obj.empty()) continue;
          Value& req = obj_at(*res, "requests");
          for (auto& m : lim->obj) set_default(req, m.k.c_str(), m.v);
        }
    default_pod_spec(spec);
  } else if (r.key == "services") {
    Value& spec = obj_at(o, "spec");
    set_default(spec, "type", Value::str("ClusterIP"));
    set_default(spec, "sessionAffinity", Value::str("None"));
    std::string type = spec.str_or("type");
    if ((type == "ClusterIP" || type == "NodePort" || type == "LoadBalancer") && spec.str_or("clusterIP") != "None") {
      Value fam = Value::array();
      fam.arr.push_back(Value::str("IPv4"));
      set_default(spec, "ipFamilies", fam);
      set_default(spec, "ipFamilyPolicy", Value::str("SingleStack"));
      set_default(spec, "internalTrafficPolicy", Value::str("Cluster"));
    }
    if (Value* ports = spec.get("ports"); ports && ports->is_arr())
      for (auto& p : ports->arr) {
        if (!p.is_obj()) continue;
        set_default(p, "protocol", Value::str("TCP"));
        const Value* tp = p.get("targetPort");
        if ((!tp || tp->is_null()) && p.get("port")) p["targetPort"] = *p.get("port");
      }
  }
}

bool defaulted_kind(const Res& r) {
  return r.key == "statefulsets.apps" || r.key == "deployments.apps" || r.key == "pods" || r.key == "services";
}

// `api`: also the kube-apiserver field defaulting (object-local; do_create runs it before
// taking the store lock and passes false here — the Service IP below reads the store)
void defaults(const Res& r, Value& o, bool api = true) {
  if (api && S.defaulting) api_defaults(r, o);
  if (r.key == "services") {
    Value& spec = o["spec"];
    if (!spec.is_obj()) spec = Value::object();
    if (!spec.get("type")) spec["type"] = Value::str("ClusterIP");
    if (spec.str_or("type") == "ClusterIP" && spec.str_or("clusterIP").empty()) {
      char ip[32];
      int64_t rvnow = S.rv.load();
      snprintf(ip, sizeof(ip), "10.96.%d.%d", (int)((rvnow >> 8) & 255), (int)((rvnow & 255) ? (rvnow & 255) : 1));
      spec["clusterIP"] = Value::str(ip);
      Value ips = Value::array();
      ips.arr.push_back(Value::str(ip));
      spec["clusterIPs"] = ips;
    }
  } else if (r.key == "namespaces") {
    Value& m = mdm(o);
    Value& labels = m["labels"];
    if (!labels.is_obj()) labels = Value::object();
    labels["kubernetes.io/metadata.name"] = Value::str(m.str_or("name"));
    if (!o.get("status")) {
      Value st = Value::object();
      st["phase"] = Value::str("Active");
      o["status"] = st;
    }
  }
}

// ------------------------------------------------------------------ admission (MutatingWebhookConfiguration)

struct Webhook {
  std::string name, url_host, url_path, ca_pem, svc_ns, svc_name, svc_path;
  int url_port = 443, svc_port = 443;
  bool fail_closed = true, has_url = false;
  double timeout_s = 10;
  Value rules;
  bool has_ns_sel = false, has_obj_sel = false;
  std::vector<LReq> ns_sel, obj_sel;
  std::vector<std::string> conditions;  // matchConditions[].expression
};

// ------------------------------------------------------------------ matchConditions (a CEL subset)
// has(<object|oldObject>.<field>...), !, &&, ||, parentheses, true and false: the expressions
// this repository's configurations use (utils/celmatch.py is the Python apiserver's twin).
// Anything else fails to compile, and a compile error evaluates as an error: failurePolicy
// decides.  CEL's logical operators absorb errors (false && err is false, true || err true).
struct CelErr {
  std::string msg;
};

struct CelNode {
  enum Kind { LIT, NOT, AND, OR, HAS } k = LIT;
  bool lit = false, old_root = false;
  std::vector<std::string> path;
  std::vector<CelNode> kids;
};

struct CelParser {
  std::string src;
  std::vector<std::string> toks;
  size_t pos = 0;

  explicit CelParser(const std::string& s) : src(s) {
    size_t i = 0;
    while (i < src.size()) {
      const char c = src[i];
      if (std::isspace((unsigned char)c)) {
        ++i;
      } else if ((c == '|' || c == '&') && i + 1 < src.size() && src[i + 1] == c) {
        toks.push_back(src.substr(i, 2));
        i += 2;
      } else if (c == '!' || c == '(' || c == ')' || c == '.') {
        toks.push_back(std::string(1, c));
        ++i;
      } else if (std::isalpha((unsigned char)c) || c == '_') {
        size_t j = i;
        while (j < src.size() && (std::isalnum((unsigned char)src[j]) || src[j] == '_')) ++j;
        toks.push_back(src.substr(i, j - i));
        i = j;
      } else {
        throw CelErr{"unsupported CEL at '" + src.substr(i) + "'"};
      }
    }
  }
  bool at(const char* t) const { return pos < toks.size() && toks[pos] == t; }
  std::string take(const char* want = nullptr) {
    if (pos >= toks.size() || (want && toks[pos] != want))
      throw CelErr{std::string("expected ") + (want ? want : "a term") + " in '" + src + "'"};
    return toks[pos++];
  }
  CelNode chain(CelNode::Kind k, const char* op, CelNode (CelParser::*next)()) {
    CelNode first = (this->*next)();
    if (!at(op)) return first;
    CelNode n;
    n.k = k;
    n.kids.push_back(std::move(first));
    while (at(op)) {
      take();
      n.kids.push_back((this->*next)());
    }
    return n;
  }
  CelNode disj() { return chain(CelNode::OR, "||", &CelParser::conj); }
  CelNode conj() { return chain(CelNode::AND, "&&", &CelParser::unary); }
  CelNode unary() {
    if (!at("!")) return primary();
    take();
    CelNode n;
    n.k = CelNode::NOT;
    n.kids.push_back(unary());
    return n;
  }
  CelNode primary() {
    const std::string t = take();
    if (t == "(") {
      CelNode e = disj();
      take(")");
      return e;
    }
    CelNode n;
    if (t == "true" || t == "false") {
      n.lit = t == "true";
      return n;
    }
    if (t != "has") throw CelErr{"unsupported CEL term '" + t + "' in '" + src + "'"};
    take("(");
    const std::string root = take();
    if (root != "object" && root != "oldObject") throw CelErr{"unsupported root '" + root + "' in '" + src + "'"};
    n.k = CelNode::HAS;
    n.old_root = root == "oldObject";
    while (at(".")) {
      take();
      const std::string f = take();
      if (!(std::isalpha((unsigned char)f[0]) || f[0] == '_')) throw CelErr{"unsupported field '" + f + "'"};
      n.path.push_back(f);
    }
    if (n.path.empty()) throw CelErr{"has() needs a field selection in '" + src + "'"};
    take(")");
    return n;
  }
  CelNode parse() {
    CelNode n = disj();
    if (pos != toks.size()) throw CelErr{"trailing tokens in '" + src + "'"};
    return n;
  }
};

bool cel_eval(const CelNode& n, const Value& obj, const Value* old) {
  switch (n.k) {
    case CelNode::LIT:
      return n.lit;
    case CelNode::NOT:
      return !cel_eval(n.kids[0], obj, old);
    case CelNode::AND:
    case CelNode::OR: {
      const bool absorbing = n.k == CelNode::OR;
      bool failed = false;
      CelErr err;
      for (const CelNode& k : n.kids) {
        try {
          if (cel_eval(k, obj, old) == absorbing) return absorbing;
        } catch (const CelErr& e) {
          failed = true;
          err = e;
        }
      }
      if (failed) throw err;
      return !absorbing;
    }
    case CelNode::HAS: {
      const Value* cur = n.old_root ? old : &obj;
      if (!cur || cur->t == T::Null) throw CelErr{std::string(n.old_root ? "oldObject" : "object") + " is null"};
      for (size_t i = 0; i + 1 < n.path.size(); ++i) {
        cur = cur->is_obj() ? cur->get(n.path[i]) : nullptr;
        if (!cur) throw CelErr{"no such key: " + n.path[i]};
      }
      if (!cur->is_obj()) throw CelErr{"has() on a non-map before " + n.path.back()};
      const Value* v = cur->get(n.path.back());
      return v && v->t != T::Null;
    }
  }
  return false;
}

// every condition true: call the webhook.  Any false: skip it.  Otherwise an error: refuse
// the request (failurePolicy Fail) or skip the webhook (Ignore)
bool conditions_allow(const Webhook& w, const Value& obj, const Value* old) {
  bool failed = false;
  std::string msg;
  for (const std::string& c : w.conditions) {
    try {
      if (!cel_eval(CelParser(c).parse(), obj, old)) return false;
    } catch (const CelErr& e) {
      failed = true;
      msg = e.msg;
    }
  }
  if (failed && w.fail_closed) throw Internal("failed calling webhook \"" + w.name + "\": matchConditions: " + msg);
  return !failed;
}

// metav1.LabelSelector (matchLabels + matchExpressions) -> requirements
std::vector<LReq> selector_reqs(const Value& sel) {
  std::vector<LReq> out;
  if (const Value* ml = sel.get("matchLabels"))
    if (ml->is_obj())
      for (auto& kv : ml->obj) out.push_back({kv.k, "=", {kv.v.s}});
  if (const Value* me = sel.get("matchExpressions"))
    if (me->is_arr())
      for (auto& e : me->arr) {
        std::string op = e.str_or("operator");
        LReq r{e.str_or("key"), op == "In" ? "in" : op == "NotIn" ? "notin" : op == "Exists" ? "exists" : "!", {}};
        if (const Value* vs = e.get("values"))
          if (vs->is_arr())
            for (auto& v : vs->arr) r.vals.push_back(v.s);
        out.push_back(r);
      }
  return out;
}

bool rule_match(const Value& rules, const Res& r, const std::string& op) {
  if (!rules.is_arr()) return false;
  auto has = [](const Value* list, const std::string& x) {
    if (!list || !list->is_arr()) return false;
    for (auto& v : list->arr)
      if (v.is_str() && (v.s == "*" || v.s == x)) return true;
    return false;
  };
  for (auto& rule : rules.arr) {
    if (!has(rule.get("operations"), op)) continue;
    if (!has(rule.get("apiGroups"), r.group)) continue;
    if (!has(rule.get("resources"), r.plural)) continue;
    return true;
  }
  return false;
}

std::string b64decode(const std::string& in) {
  static int T_[256];
  static bool init = false;
  if (!init) {
    for (int& x : T_) x = -1;
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int k = 0; k < 64; ++k) T_[(unsigned char)a[k]] = k;
    init = true;
  }
  std::string out;
  int val = 0, bits = -8;
  for (unsigned char c : in) {
    if (T_[c] == -1) continue;
    val = (val << 6) + T_[c];
    bits += 6;
    if (bits >= 0) {
      out += (char)((val >> bits) & 0xFF);
      bits -= 8;
    }
  }
  return out;
}

std::vector<Webhook> webhooks_for(const Res& r, const std::string& op) {
  std::vector<Webhook> out;
  Res* mwc = by_kind("admissionregistration.k8s.io", "MutatingWebhookConfiguration");
  if (!mwc) return out;
  std::vector<Obj> cfgs;
  {
    StoreLock g(bucket(*mwc));
    for (auto& kv : bucket(*mwc).objs) cfgs.push_back(kv.second);
  }
  for (auto& c : cfgs) {
    const Value* whs = c->get("webhooks");
    if (!whs || !whs->is_arr()) continue;
    for (auto& wh : whs->arr) {
      const Value* rules = wh.get("rules");
      if (!rules || !rule_match(*rules, r, op)) continue;
      Webhook w;
      w.name = wh.str_or("name");
      w.fail_closed = wh.str_or("failurePolicy", "Fail") == "Fail";
      const Value* ts = wh.get("timeoutSeconds");
      if (ts && ts->t == T::Int) w.timeout_s = (double)ts->i;
      if (const Value* ns = wh.get("namespaceSelector"))
        if (ns->is_obj() && !ns->obj.empty()) {
          w.has_ns_sel = true;
          w.ns_sel = selector_reqs(*ns);
        }
      if (const Value* os = wh.get("objectSelector"))
        if (os->is_obj() && !os->obj.empty()) {
          w.has_obj_sel = true;
          w.obj_sel = selector_reqs(*os);
        }
      if (const Value* mc = wh.get("matchConditions"))
        if (mc->is_arr())
          for (auto& c : mc->arr) w.conditions.push_back(c.str_or("expression"));
      const Value* cc = wh.get("clientConfig");
      if (cc) {
        std::string ca = cc->str_or("caBundle");
        if (!ca.empty()) w.ca_pem = b64decode(ca);
        std::string url = cc->str_or("url");
        if (!url.empty()) {
          w.has_url = true;
          std::string rest = url.substr(url.find("://") + 3);
          size_t slash = rest.find('/');
          std::string hostport = rest.substr(0, slash);
          w.url_path = slash == std::string::npos ? "/" : rest.substr(slash);
          size_t colon = hostport.rfind(':');
          w.url_host = colon == std::string::npos ? hostport : hostport.substr(0, colon);
          w.url_port = colon == std::string::npos ? 443 : std::stoi(hostport.substr(colon + 1));
        } else if (const Value* svc = cc->get("service")) {
          w.svc_ns = svc->str_or("namespace");
          w.svc_name = svc->str_or("name");
          w.svc_path = svc->str_or("path", "/");
          const Value* p = svc->get("port");
          if (p && p->t == T::Int) w.svc_port = (int)p->i;
        }
      }
      out.push_back(std::move(w));
    }
  }
  return out;
}

std::atomic<uint64_t> g_rr{0};

// Service → Endpoints (round robin over ready addresses) like a ClusterIP Service would.
bool resolve_service(const Webhook& w, std::string* host, int* port) {
  Res* ep = by_kind("", "Endpoints");
  if (!ep) return false;
  Obj o;
  {
    StoreLock g(bucket(*ep));
    auto it = bucket(*ep).objs.find({w.svc_ns, w.svc_name});
    if (it == bucket(*ep).objs.end()) return false;
    o = it->second;
  }
  std::vector<std::pair<std::string, int>> targets;
  const Value* subsets = o->get("subsets");
  if (!subsets || !subsets->is_arr()) return false;
  for (auto& ss : subsets->arr) {
    const Value* addrs = ss.get("addresses");
    const Value* ports = ss.get("ports");
    if (!addrs || !addrs->is_arr() || !ports || !ports->is_arr() || ports->arr.empty()) continue;
    int p = 0;
    for (auto& pp : ports->arr) {
      const Value* pv = pp.get("port");
      if (pv && pv->t == T::Int) {
        p = (int)pv->i;
        break;
      }
    }
    for (auto& a : addrs->arr) targets.push_back({a.str_or("ip"), p});
  }
  if (targets.empty()) return false;
  auto& t = targets[g_rr++ % targets.size()];
  *host = t.first;
  *port = t.second;
  return true;
}

struct TlsConn {
  int fd = -1;
  SSL* ssl = nullptr;
  ~TlsConn() {
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
    }
    if (fd >= 0) close(fd);
  }
};

std::mutex g_ctx_mu;
std::map<std::string, SSL_CTX*> g_ctx;  // caBundle → context

SSL_CTX* ctx_for(const std::string& ca_pem) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  auto it = g_ctx.find(ca_pem);
  if (it != g_ctx.end()) return it->second;
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  if (!ca_pem.empty()) {
    BIO* bio = BIO_new_mem_buf(ca_pem.data(), (int)ca_pem.size());
    X509_STORE* st = SSL_CTX_get_cert_store(ctx);
    while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
      X509_STORE_add_cert(st, x);
      X509_free(x);
    }
    ERR_clear_error();
    BIO_free(bio);
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
  } else {
    SSL_CTX_set_default_verify_paths(ctx);
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
  }
  g_ctx[ca_pem] = ctx;
  return ctx;
}

// connection pool: host:port|ca -> idle connections
// Connections to each webhook endpoint: idle ones are reused (keep-alive), and at most
// g_webhook_conns are open at once — kube-apiserver multiplexes its admission calls over one
// HTTP/2 connection, so a burst of creates must not turn into a burst of TLS handshakes
// against the webhook server; a call finding them all busy waits for one to come back.
struct WebhookPool {
  std::vector<std::unique_ptr<TlsConn>> idle;
  int open = 0;
};
std::mutex g_pool_mu;
std::condition_variable g_pool_cv;
std::map<std::string, WebhookPool> g_pool;
int g_webhook_conns = 16;

std::unique_ptr<TlsConn> tls_connect(const std::string& host, int port, const std::string& ca, double timeout_s) {
  auto c = std::make_unique<TlsConn>();
  const uint64_t t0 = mono_ns();
  struct addrinfo hints {};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("cannot resolve " + host);
  c->fd = socket(res->ai_family, SOCK_STREAM, 0);
  struct timeval tv;
  tv.tv_sec = (long)timeout_s;
  tv.tv_usec = (long)((timeout_s - (long)timeout_s) * 1e6);
  setsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(c->fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int one = 1;
  setsockopt(c->fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int rc = connect(c->fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc != 0) throw std::runtime_error("connect failed to " + host + ":" + std::to_string(port));
  c->ssl = SSL_new(ctx_for(ca));
  SSL_set_fd(c->ssl, c->fd);
  X509_VERIFY_PARAM* param = SSL_get0_param(c->ssl);
  struct in_addr a4;
  if (inet_pton(AF_INET, host.c_str(), &a4) == 1) {
    X509_VERIFY_PARAM_set1_ip_asc(param, host.c_str());
  } else {
    SSL_set_tlsext_host_name(c->ssl, host.c_str());
    X509_VERIFY_PARAM_set1_host(param, host.c_str(), 0);
  }
  if (SSL_connect(c->ssl) != 1) {
    unsigned long e = ERR_get_error();
    char buf[256];
    ERR_error_string_n(e, buf, sizeof(buf));
    throw std::runtime_error(std::string("TLS handshake failed: ") + buf);
  }
  P.webhook_dials++;
  P.webhook_dial_ns += mono_ns() - t0;
  return c;
}

bool tls_write_all(TlsConn& c, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    int n = SSL_write(c.ssl, s.data() + off, (int)(s.size() - off));
    if (n <= 0) return false;
    off += n;
  }
  return true;
}

// minimal HTTP/1.1 response reader (Content-Length or chunked); *close: the server will
// close the connection after this response (Connection: close), so it is not pooled
bool tls_read_response(TlsConn& c, int* status, std::string* body, bool* close = nullptr) {
  std::string buf;
  char tmp[16384];
  size_t hdr_end;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    int n = SSL_read(c.ssl, tmp, sizeof(tmp));
    if (n <= 0) return false;
    buf.append(tmp, n);
  }
  std::string head = buf.substr(0, hdr_end);
  std::string rest = buf.substr(hdr_end + 4);
  *status = std::atoi(head.c_str() + head.find(' ') + 1);
  std::string lower = head;
  std::transform(lower.begin(), lower.end(), lower.begin(), ::tolower);
  if (close) *close = lower.find("connection: close") != std::string::npos;
  size_t cl = lower.find("content-length:");
  if (cl != std::string::npos) {
    size_t len = std::stoul(lower.substr(cl + 15));
    while (rest.size() < len) {
      int n = SSL_read(c.ssl, tmp, sizeof(tmp));
      if (n <= 0) return false;
      rest.append(tmp, n);
    }
    *body = rest.substr(0, len);
    return true;
  }
  if (lower.find("transfer-encoding: chunked") != std::string::npos) {
    std::string out;
    while (true) {
      size_t le;
      while ((le = rest.find("\r\n")) == std::string::npos) {
        int n = SSL_read(c.ssl, tmp, sizeof(tmp));
        if (n <= 0) return false;
        rest.append(tmp, n);
      }
      size_t sz = std::stoul(rest.substr(0, le), nullptr, 16);
      rest.erase(0, le + 2);
      while (rest.size() < sz + 2) {
        int n = SSL_read(c.ssl, tmp, sizeof(tmp));
        if (n <= 0) return false;
        rest.append(tmp, n);
      }
      if (sz == 0) break;
      out.append(rest, 0, sz);
      rest.erase(0, sz + 2);
    }
    *body = out;
    return true;
  }
  return false;
}

Value call_webhook(const Webhook& w, const Value& review) {
  std::string host = w.url_host, path = w.url_path;
  int port = w.url_port;
  if (!w.has_url) {
    if (!resolve_service(w, &host, &port)) throw std::runtime_error("no endpoints for service " + w.svc_ns + "/" + w.svc_name);
    path = w.svc_path;
  }
  std::string body = kj::dump(review);
  std::string req = "POST " + path + " HTTP/1.1\r\nHost: " + host + ":" + std::to_string(port) +
                    "\r\nContent-Type: application/json\r\nAccept: application/json\r\nContent-Length: " +
                    std::to_string(body.size()) + "\r\n\r\n" + body;
  std::string pool_key = host + ":" + std::to_string(port) + "|" + w.ca_pem;
  // a slot (an idle connection, or room to open one) for the duration of the call
  auto acquire = [&](bool allow_idle) -> std::unique_ptr<TlsConn> {
    std::unique_lock<std::mutex> g(g_pool_mu);
    auto deadline = std::chrono::system_clock::now() + std::chrono::milliseconds((int64_t)(w.timeout_s * 1000));
    while (true) {
      WebhookPool& p = g_pool[pool_key];
      if (allow_idle && !p.idle.empty()) {
        auto c = std::move(p.idle.back());
        p.idle.pop_back();
        return c;
      }
      if (p.open < g_webhook_conns) {
        p.open++;
        return nullptr;  // the caller opens one
      }
      if (g_pool_cv.wait_until(g, deadline) == std::cv_status::timeout)
        throw std::runtime_error("timed out waiting for a connection to the webhook");
    }
  };
  auto give_back = [&](std::unique_ptr<TlsConn> c) {  // nullptr: the slot's connection is gone
    {
      std::lock_guard<std::mutex> g(g_pool_mu);
      WebhookPool& p = g_pool[pool_key];
      if (c) p.idle.push_back(std::move(c));
      else p.open--;
    }
    g_pool_cv.notify_one();
  };
  for (int attempt = 0; attempt < 2; ++attempt) {
    const uint64_t t0 = mono_ns();
    std::unique_ptr<TlsConn> c = acquire(attempt == 0);
    bool reused = (bool)c;
    const uint64_t t1 = mono_ns();
    if (!c) {
      try {
        c = tls_connect(host, port, w.ca_pem, w.timeout_s);
      } catch (...) {
        give_back(nullptr);
        throw;
      }
    }
    const uint64_t t2 = mono_ns();
    int status = 0;
    std::string resp;
    bool close = false;
    const bool ok = tls_write_all(*c, req) && tls_read_response(*c, &status, &resp, &close);
    if (g_stall_ms > 0 && mono_ns() - t0 >= (uint64_t)g_stall_ms * 1000000ull) {
      timespec ts;
      clock_gettime(CLOCK_REALTIME, &ts);
      fprintf(stderr, "stall-watchdog: webhook call %.1f ms (slot %.1f, %s %.1f, round trip %.1f, attempt %d, ok %d) ending at %.6f\n",
              (mono_ns() - t0) / 1e6, (t1 - t0) / 1e6, reused ? "pooled" : "dial", (t2 - t1) / 1e6,
              (mono_ns() - t2) / 1e6, attempt, (int)ok, (double)ts.tv_sec + ts.tv_nsec / 1e9);
    }
    if (ok) {
      if (close) c.reset();  // the webhook hangs up after this answer: the slot reconnects next time
      give_back(std::move(c));
      if (status != 200) throw std::runtime_error("webhook returned HTTP " + std::to_string(status));
      return kj::parse(resp);
    }
    c.reset();
    give_back(nullptr);
    if (!reused) throw std::runtime_error("webhook request failed");
  }
  throw std::runtime_error("webhook request failed");
}

// namespaceSelector / objectSelector of a webhook against the object being admitted
bool selectors_match(const Webhook& w, const Res& r, const Value& obj, const Value* old) {
  if (w.has_obj_sel && !match_labels(w.obj_sel, obj) && !(old && match_labels(w.obj_sel, *old))) return false;
  if (!w.has_ns_sel) return true;
  if (r.kind == "Namespace" && r.group.empty()) return match_labels(w.ns_sel, obj);
  if (!r.namespaced) return true;  // cluster-scoped objects are not subject to namespaceSelector
  Res* nsr = by_kind("", "Namespace");
  Obj ns;
  if (nsr) {
    StoreLock g(bucket(*nsr));
    auto it = bucket(*nsr).objs.find({"", mget(obj, "namespace")});
    if (it != bucket(*nsr).objs.end()) ns = it->second;
  }
  if (ns) return match_labels(w.ns_sel, *ns);
  Value stub = Value::object();  // unknown namespace: only the implicit name label
  Value m = Value::object();
  Value l = Value::object();
  l["kubernetes.io/metadata.name"] = Value::str(mget(obj, "namespace"));
  m["labels"] = l;
  stub["metadata"] = m;
  return match_labels(w.ns_sel, stub);
}

Value admit(const char* op, const Res& r, Value obj, const Value* old) {
  PhaseTimer pt(PH_ADMIT);
  auto hooks = webhooks_for(r, op);
  for (auto& w : hooks) {
    if (!selectors_match(w, r, obj, old)) continue;
    if (!w.conditions.empty() && !conditions_allow(w, obj, old)) continue;
    Value review = Value::object();
    review["apiVersion"] = Value::str("admission.k8s.io/v1");
    review["kind"] = Value::str("AdmissionReview");
    Value req = Value::object();
    req["uid"] = Value::str(uuid4());
    req["operation"] = Value::str(op);
    req["name"] = Value::str(mget(obj, "name"));
    req["namespace"] = Value::str(mget(obj, "namespace"));
    Value kind = Value::object();
    kind["group"] = Value::str(r.group);
    kind["version"] = Value::str(r.storage);
    kind["kind"] = Value::str(r.kind);
    req["kind"] = kind;
    Value res = Value::object();
    res["group"] = Value::str(r.group);
    res["version"] = Value::str(r.storage);
    res["resource"] = Value::str(r.plural);
    req["resource"] = res;
    req["object"] = obj;
    req["oldObject"] = old ? *old : Value();
    review["request"] = std::move(req);
    S.webhook_calls++;
    Value out;
    uint64_t t_admit = mono_ns();
    struct AdmitTimer {
      uint64_t t0;
      ~AdmitTimer() {
        uint64_t d = mono_ns() - t0;
        P.admit_wall_ns += d;
        uint64_t i = g_admit.seq.fetch_add(1);
        g_admit.us[i & (kAdmitRing - 1)].store((uint32_t)std::min<uint64_t>(d / 1000, 0xffffffffu));
      }
    } admit_timer{t_admit};
    try {
      out = call_webhook(w, review);
    } catch (const std::exception& e) {
      if (w.fail_closed) throw Internal("failed calling webhook \"" + w.name + "\": " + e.what());
      continue;
    }
    const Value* resp = out.get("response");
    if (!resp) {
      if (w.fail_closed) throw Internal("webhook \"" + w.name + "\" returned no response");
      continue;
    }
    const Value* allowed = resp->get("allowed");
    if (!allowed || allowed->t != T::Bool || !allowed->b) {
      const Value* st = resp->get("status");
      throw Internal("admission webhook \"" + w.name + "\" denied the request: " + (st ? st->str_or("message") : ""));
    }
    std::string p = resp->str_or("patch");
    if (!p.empty()) {
      try {
        obj = apply_json_patch(std::move(obj), kj::parse(b64decode(p)));
      } catch (const PatchErr& e) {
        throw Internal("webhook \"" + w.name + "\" returned an invalid patch: " + e.msg);
      }
    }
  }
  return obj;
}

// ------------------------------------------------------------------ store operations

Res& res_checked(Res* r) {
  if (!r->installed) throw NoKindMatch(r->kind);
  return *r;
}

std::pair<std::vector<Obj>, int64_t> do_list(const Res& r, const std::string& ns, const std::string& lsel,
                                             const std::string& fsel) {
  auto lr = parse_labels(lsel);
  auto fr = parse_fields(fsel);
  std::vector<Obj> out;
  Bucket& b = bucket(r);
  StoreLock g(b);  // the list's resourceVersion: no commit of this resource is in flight
  if (!ns.empty() && r.namespaced) {
    for (auto it = b.objs.lower_bound({ns, ""}); it != b.objs.end() && it->first.first == ns; ++it)
      if ((lr.empty() || match_labels(lr, *it->second)) && (fr.empty() || match_fields(fr, *it->second)))
        out.push_back(it->second);
  } else {
    for (auto& kv : b.objs)
      if ((lr.empty() || match_labels(lr, *kv.second)) && (fr.empty() || match_fields(fr, *kv.second)))
        out.push_back(kv.second);
  }
  return {out, S.rv.load()};
}

Obj do_get(const Res& r, const std::string& ns, const std::string& name) {
  Bucket& b = bucket(r);
  StoreLock g(b);
  auto it = b.objs.find({r.namespaced ? ns : "", name});
  if (it == b.objs.end()) throw NotFound(r.err_res(), name);
  return it->second;
}

void remove_locked(const Res& r, Obj live, Obj final);
void gc_dependents(const std::string& owner_uid);
void sync_delete_locked(const Res& r, const std::string& ns, const std::string& name);

Obj do_create(const Res& r, const std::string& url_ns, Value obj, bool dry) {
  Value& m = mdm(obj);
  std::string ns;
  if (r.namespaced) {
    ns = m.str_or("namespace");
    if (ns.empty()) ns = url_ns;
    if (ns.empty()) throw BadRequest("the namespace of the object must be set");
    if (!url_ns.empty() && !m.str_or("namespace").empty() && url_ns != m.str_or("namespace"))
      throw BadRequest("the namespace of the provided object does not match the namespace sent on the request");
    m["namespace"] = Value::str(ns);
  } else {
    m.erase("namespace");
  }
  if (!m.str_or("resourceVersion").empty()) throw BadRequest("resourceVersion should not be set on objects to be created");
  if (m.str_or("name").empty()) {
    std::string gen = m.str_or("generateName");
    if (gen.empty()) throw Invalid(r.kind, "", "metadata.name: Required value: name or generateName is required");
    m["name"] = Value::str(gen + rand_suffix());
  }
  obj["apiVersion"] = Value::str(r.api_version(r.storage));
  obj = admit("CREATE", r, std::move(obj), nullptr);
  if (auto err = validate(r, obj)) throw Invalid(r.group.empty() ? r.singular : r.kind + "." + r.group, mget(obj, "name"), *err);
  {
    Value& mm = mdm(obj);
    mm["uid"] = Value::str(uuid4());
    mm["creationTimestamp"] = Value::str(rfc3339_now());
    mm.erase("deletionTimestamp");
    if (obj.get("spec") || r.status) mm["generation"] = Value::integer(1);
    if (r.status && !r.group.empty()) obj.erase("status");
  }
  std::pair<std::string, std::string> k{ns, mget(obj, "name")};
  if (S.defaulting) api_defaults(r, obj);  // object-local: outside the store lock
  if (!dry) storage_latency();
  Bucket& b = bucket(r);
  StoreLock g(b);
  if (b.objs.count(k)) throw AlreadyExists(r.err_res(), k.second);
  defaults(r, obj, false);
  if (dry) return std::make_shared<const Value>(std::move(obj));
  mdm(obj)["resourceVersion"] = Value::str(std::to_string(++S.rv));
  auto sp = std::make_shared<const Value>(std::move(obj));
  b.objs[k] = sp;
  {
    const std::string u = mget(*sp, "uid");
    IdxStripe& st = idx(u);
    std::lock_guard<std::mutex> ig(st.mu);
    st.uids[u] = std::make_tuple(r.key, ns, k.second);
  }
  index_owner(r, *sp, false);
  S.writes++;
  emit(r, "ADDED", sp, nullptr);
  // the GC's "absent owner" rule: a dependent created after all of its owners are gone
  // (a controller acting on a stale cache) is collected right away
  if (S.gc) {
    const Value* refs = md(*sp)->get("ownerReferences");
    if (refs && refs->is_arr() && !refs->arr.empty()) {
      bool live = false;
      for (auto& ref : refs->arr) {
        std::string av = ref.str_or("apiVersion");
        auto slash = av.find('/');
        Res* owner = by_kind(slash == std::string::npos ? "" : av.substr(0, slash), ref.str_or("kind"));
        // an owner of a kind this server does not serve cannot be verified: keep the object
        const std::string u = ref.str_or("uid");
        IdxStripe& st = idx(u);
        std::lock_guard<std::mutex> ig(st.mu);
        if (!owner || st.uids.count(u)) live = true;
      }
      if (!live) {
        sync_delete_locked(r, ns, k.second);
        return sp;
      }
    }
  }
  return sp;
}

// nw's server-owned metadata from `base` (the version it replaces); generation bumped
// when the spec changes; no new finalizers once deletion has started
void prepare_update(const Res& r, const Value& base, Value& nw) {
  Value& m = mdm(nw);
  const Value& lm = *md(base);
  std::string ns = mget(base, "namespace"), name = mget(base, "name");
  for (const char* k : {"uid", "creationTimestamp", "deletionTimestamp", "deletionGracePeriodSeconds"}) {
    const Value* v = lm.get(k);
    if (v) m[k] = *v;
    else m.erase(k);
  }
  if (r.namespaced) m["namespace"] = Value::str(ns);
  else m.erase("namespace");
  m["name"] = Value::str(name);
  if (lm.get("deletionTimestamp")) {
    std::set<std::string> before, added;
    if (const Value* f = lm.get("finalizers"))
      for (auto& x : f->arr) before.insert(x.s);
    if (const Value* f = m.get("finalizers"))
      for (auto& x : f->arr)
        if (!before.count(x.s)) added.insert(x.s);
    if (!added.empty()) {
      std::string l;
      for (auto& a : added) l += (l.empty() ? "" : " ") + a;
      throw Forbidden("no new finalizers can be added if the object is being deleted, found new finalizers [" + l + "]");
    }
  }
  if (S.defaulting && defaulted_kind(r)) {
    api_defaults(r, nw);
    if (r.key == "services") {  // the allocated ClusterIP is immutable
      const Value* bs = base.get("spec");
      Value& ns_ = obj_at(nw, "spec");
      for (const char* k : {"clusterIP", "clusterIPs"}) {
        const Value* have = ns_.get(k);
        const Value* was = bs ? bs->get(k) : nullptr;
        if (was && (!have || have->is_null() || (have->is_str() && have->s.empty()))) ns_[k] = *was;
      }
    }
  }
  if (const Value* gen = lm.get("generation")) {
    int64_t gv = gen->i;
    if (!spec_equal(nw, base)) gv++;
    m["generation"] = Value::integer(gv);
  }
  m["resourceVersion"] = Value::str(mget(base, "resourceVersion"));
}

// Commit a new version over `cur` (caller holds no lock).  The update is prepared and
// compared against the snapshot `cur` OUTSIDE the store lock; when the stored object is
// still that snapshot at commit time (the common case) the lock covers only the commit
// itself — resourceVersion, the map slot, the owner index and the watch event.
Obj commit_update(const Res& r, const Obj& cur, Value nw) {
  const std::string want_rv = mdm(nw).str_or("resourceVersion");
  const std::string ns = mget(*cur, "namespace"), name = mget(*cur, "name");
  bool noop;
  {
    PhaseTimer pt(PH_PREPARE);
    prepare_update(r, *cur, nw);
    noop = equal_except_meta(nw, *cur);
  }
  if (!noop) storage_latency();
  Bucket& b = bucket(r);
  StoreLock g(b);
  auto it = b.objs.find({ns, name});
  if (it == b.objs.end()) throw NotFound(r.err_res(), name);
  Obj live = it->second;
  if (!want_rv.empty() && want_rv != mget(*live, "resourceVersion")) throw Conflict(r.err_res(), name);
  if (live != cur) {  // written since the snapshot: prepare against the live version
    prepare_update(r, *live, nw);
    noop = equal_except_meta(nw, *live);
  }
  if (noop) return live;  // no-op write
  const Value* fin = md(nw)->get("finalizers");
  bool no_fin = !fin || !fin->is_arr() || fin->arr.empty();
  if (md(*live)->get("deletionTimestamp") && no_fin) {
    mdm(nw)["resourceVersion"] = Value::str(std::to_string(++S.rv));
    auto out = std::make_shared<const Value>(std::move(nw));
    remove_locked(r, live, out);
    return out;
  }
  mdm(nw)["resourceVersion"] = Value::str(std::to_string(++S.rv));
  index_owner(r, *live, true);
  auto sp = std::make_shared<const Value>(std::move(nw));
  it->second = sp;
  index_owner(r, *sp, false);
  S.writes++;
  emit(r, "MODIFIED", sp, live);
  return sp;
}

Obj do_update(const Res& r, const std::string& ns, const std::string& name, Value nw, const std::string& sub) {
  Obj cur;
  {
    StoreLock g(bucket(r));
    auto it = bucket(r).objs.find({r.namespaced ? ns : "", name});
    if (it == bucket(r).objs.end()) throw NotFound(r.err_res(), name);
    cur = it->second;
  }
  nw["apiVersion"] = Value::str(r.api_version(r.storage));
  if (sub == "status") {
    Value merged = *cur;
    if (const Value* st = nw.get("status")) merged["status"] = *st;
    else merged.erase("status");
    mdm(merged)["resourceVersion"] = Value::str(mget(nw, "resourceVersion"));
    nw = std::move(merged);
    if (auto err = validate(r, nw)) throw Invalid(r.kind + "." + r.group, name, *err);
  } else {
    if (r.status) {
      if (const Value* st = cur->get("status")) nw["status"] = *st;
      else nw.erase("status");
    }
    nw = admit("UPDATE", r, std::move(nw), cur.get());
    if (auto err = validate(r, nw)) throw Invalid(r.kind + "." + r.group, name, *err);
  }
  return commit_update(r, cur, std::move(nw));
}

Obj do_patch_once(const Res& r, const std::string& ns, const std::string& name, const Value& patch,
                    const std::string& ptype, const std::string& sub) {
  Obj cur;
  {
    StoreLock g(bucket(r));
    auto it = bucket(r).objs.find({r.namespaced ? ns : "", name});
    if (it == bucket(r).objs.end()) throw NotFound(r.err_res(), name);
    cur = it->second;
  }
  Value nw;
  try {
    PhaseTimer pt(PH_PATCH);
    if (ptype == "merge") nw = merge_patch(*cur, patch);
    else if (ptype == "json") nw = apply_json_patch(*cur, patch);
    else if (ptype == "strategic") nw = strategic_patch(*cur, patch);
    else throw BadRequest("unsupported patch type " + ptype);
  } catch (const PatchErr& e) {
    throw Invalid(r.kind, name, e.msg);
  }
  const Value* pm = patch.is_obj() ? patch.get("metadata") : nullptr;
  bool precond = pm && pm->is_obj() && !pm->str_or("resourceVersion").empty();
  if (!precond) mdm(nw)["resourceVersion"] = Value::str(mget(*cur, "resourceVersion"));
  if (sub == "status") {
    Value merged = *cur;
    const Value* st = nw.get("status");
    merged["status"] = st ? *st : Value();
    mdm(merged)["resourceVersion"] = Value::str(mget(nw, "resourceVersion"));
    nw = std::move(merged);
    if (auto err = validate(r, nw)) throw Invalid(r.kind + "." + r.group, name, *err);
  } else {
    if (r.status) {
      if (const Value* st = cur->get("status")) nw["status"] = *st;
      else nw.erase("status");
    }
    nw = admit("UPDATE", r, std::move(nw), cur.get());
    if (auto err = validate(r, nw)) throw Invalid(r.kind + "." + r.group, name, *err);
  }
  return commit_update(r, cur, std::move(nw));
}

// A patch without a resourceVersion precondition applies to whatever is current: like
// the apiserver's GuaranteedUpdate loop, a conflict with a concurrent writer (e.g. during
// a slow admission webhook call) re-reads and re-applies instead of failing.
Obj do_patch(const Res& r, const std::string& ns, const std::string& name, const Value& patch,
               const std::string& ptype, const std::string& sub) {
  const Value* pm = patch.is_obj() ? patch.get("metadata") : nullptr;
  bool precond = pm && pm->is_obj() && !pm->str_or("resourceVersion").empty();
  for (int attempt = 0;; ++attempt) {
    try {
      return do_patch_once(r, ns, name, patch, ptype, sub);
    } catch (const ApiErr& e) {
      if (e.reason != "Conflict" || precond || attempt >= 16) throw;
    }
  }
}

void remove_locked(const Res& r, Obj live, Obj fp) {
  std::string ns = mget(*live, "namespace"), name = mget(*live, "name"), uid = mget(*live, "uid");
  bucket(r).objs.erase({ns, name});
  {
    IdxStripe& st = idx(uid);
    std::lock_guard<std::mutex> ig(st.mu);
    st.uids.erase(uid);
  }
  index_owner(r, *live, true);
  S.writes++;
  emit(r, "DELETED", fp, live);
  if (S.gc) t_gc.push_back(uid);  // cascaded once the lock is released (run_gc)
  // foreground owners waiting for their last dependent: re-checked after the commit, each
  // under its own resource's lock (fg_recheck)
  if (S.gc) {
    const Value* refs = md(*fp) ? md(*fp)->get("ownerReferences") : nullptr;
    if (refs && refs->is_arr())
      for (auto& ref : refs->arr) {
        std::string u = ref.str_or("uid");
        if (!u.empty()) t_fg.push_back(u);
      }
  }
}

// An owner being deleted in the foreground loses its "foregroundDeletion" finalizer once
// its last dependent is gone (and is removed if that was its last finalizer).
void fg_recheck(const std::string& u) {
  std::tuple<std::string, std::string, std::string> loc;
  {
    IdxStripe& st = idx(u);
    std::lock_guard<std::mutex> ig(st.mu);
    auto it = st.uids.find(u);
    if (it == st.uids.end() || st.owners.count(u)) return;
    loc = it->second;
  }
  Res* orr = by_key(std::get<0>(loc));
  if (!orr) return;
  Bucket& b = bucket(*orr);
  StoreLock g(b);
  auto it = b.objs.find({std::get<1>(loc), std::get<2>(loc)});
  if (it == b.objs.end() || mget(*it->second, "uid") != u) return;
  {
    IdxStripe& st = idx(u);
    std::lock_guard<std::mutex> ig(st.mu);
    if (st.owners.count(u)) return;  // a dependent appeared meanwhile
  }
  const Value* f = md(*it->second)->get("finalizers");
  bool fg = false;
  if (f && f->is_arr())
    for (auto& x : f->arr)
      if (x.s == "foregroundDeletion") fg = true;
  if (!fg) return;
  Value nw = *it->second;
  Value nf = Value::array();
  for (auto& x : f->arr)
    if (x.s != "foregroundDeletion") nf.arr.push_back(x);
  mdm(nw)["finalizers"] = nf;
  mdm(nw)["resourceVersion"] = Value::str(std::to_string(++S.rv));
  Obj old = it->second;
  if (nf.arr.empty()) {
    remove_locked(*orr, old, std::make_shared<const Value>(std::move(nw)));
  } else {
    auto sp = std::make_shared<const Value>(std::move(nw));
    it->second = sp;
    emit(*orr, "MODIFIED", sp, old);
  }
}

void sync_delete_locked(const Res& r, const std::string& ns, const std::string& name) {
  auto it = bucket(r).objs.find({ns, name});
  if (it == bucket(r).objs.end()) return;
  Obj cur = it->second;
  const Value* f = md(*cur)->get("finalizers");
  if (f && f->is_arr() && !f->arr.empty()) {
    if (md(*cur)->get("deletionTimestamp")) return;
    Value nw = *cur;
    mdm(nw)["deletionTimestamp"] = Value::str(rfc3339_now());
    mdm(nw)["resourceVersion"] = Value::str(std::to_string(++S.rv));
    auto sp = std::make_shared<const Value>(std::move(nw));
    it->second = sp;
    emit(r, "MODIFIED", sp, cur);
    return;
  }
  Value final = *cur;
  mdm(final)["resourceVersion"] = Value::str(std::to_string(++S.rv));
  remove_locked(r, cur, std::make_shared<const Value>(std::move(final)));
}

// Background cascade for a removed (or foreground-deleting) owner: each dependent whose
// other owners are all gone is deleted, under its own resource's lock (no lock held here).
void gc_dependents(const std::string& owner_uid) {
  std::set<std::tuple<std::string, std::string, std::string>> deps;
  {
    IdxStripe& st = idx(owner_uid);
    std::lock_guard<std::mutex> ig(st.mu);
    auto it = st.owners.find(owner_uid);
    if (it == st.owners.end()) return;
    deps = it->second;
  }
  for (auto& d : deps) {
    Res* r = by_key(std::get<0>(d));
    if (!r) continue;
    Bucket& b = bucket(*r);
    StoreLock g(b);  // its release does not recurse (t_gc_running); new owners queue up
    auto oit = b.objs.find({std::get<1>(d), std::get<2>(d)});
    if (oit == b.objs.end()) continue;
    bool other_live = false;
    if (const Value* refs = md(*oit->second)->get("ownerReferences")) {
      for (auto& ref : refs->arr) {
        std::string u = ref.str_or("uid");
        if (u == owner_uid) continue;
        IdxStripe& st = idx(u);
        std::lock_guard<std::mutex> ig(st.mu);
        if (st.uids.count(u)) other_live = true;
      }
    }
    if (other_live) continue;
    sync_delete_locked(*r, std::get<1>(d), std::get<2>(d));
  }
}

void run_gc() noexcept {
  t_gc_running = true;
  while (!t_gc.empty() || !t_fg.empty()) {
    std::vector<std::string> uids, fgs;
    uids.swap(t_gc);
    fgs.swap(t_fg);
    for (auto& u : uids) {
      try {
        gc_dependents(u);
      } catch (...) {
        // a dependent that vanished meanwhile: nothing left to collect for it
      }
    }
    for (auto& u : fgs) {
      try {
        fg_recheck(u);
      } catch (...) {
      }
    }
  }
  t_gc_running = false;
}

Value do_delete(const Res& r, const std::string& ns_, const std::string& name, const Value& opts) {
  std::string ns = r.namespaced ? ns_ : "";
  storage_latency();
  StoreLock g(bucket(r));
  auto it = bucket(r).objs.find({ns, name});
  if (it == bucket(r).objs.end()) throw NotFound(r.err_res(), name);
  Obj cur = it->second;
  if (const Value* pc = opts.get("preconditions")) {
    std::string u = pc->str_or("uid"), rv = pc->str_or("resourceVersion");
    if (!u.empty() && u != mget(*cur, "uid")) throw Conflict(r.err_res(), name, "Precondition failed: UID in precondition does not match");
    if (!rv.empty() && rv != mget(*cur, "resourceVersion")) throw Conflict(r.err_res(), name, "Precondition failed: resourceVersion does not match");
  }
  Value fins = Value::array();
  if (const Value* f = md(*cur)->get("finalizers"))
    if (f->is_arr()) fins = *f;
  std::string prop = opts.str_or("propagationPolicy", "Background");
  bool has_fg = false;
  for (auto& x : fins.arr)
    if (x.s == "foregroundDeletion") has_fg = true;
  if (prop == "Foreground" && S.gc && !has_fg) fins.arr.push_back(Value::str("foregroundDeletion"));
  if (!fins.arr.empty()) {
    if (md(*cur)->get("deletionTimestamp")) return *cur;
    Value nw = *cur;
    Value& m = mdm(nw);
    m["finalizers"] = fins;
    m["deletionTimestamp"] = Value::str(rfc3339_now());
    m["deletionGracePeriodSeconds"] = Value::integer(0);
    if (Value* gen = m.get("generation")) gen->i += 1;
    m["resourceVersion"] = Value::str(std::to_string(++S.rv));
    auto sp = std::make_shared<const Value>(std::move(nw));
    it->second = sp;
    S.writes++;
    emit(r, "MODIFIED", sp, cur);
    bool fg = false;
    for (auto& x : fins.arr)
      if (x.s == "foregroundDeletion") fg = true;
    if (fg) t_gc.push_back(mget(*cur, "uid"));  // dependents first, after this commit (run_gc)
    return *sp;
  }
  Value final = *cur;
  mdm(final)["resourceVersion"] = Value::str(std::to_string(++S.rv));
  Value out = final;
  remove_locked(r, cur, std::make_shared<const Value>(std::move(final)));
  return out;
}

// ------------------------------------------------------------------ HTTP server

std::string g_token;
std::atomic<bool> g_stop{false};

struct Conn {
  int fd;
  std::string buf;
};

bool write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
    if (w <= 0) return false;
    p += w;
    n -= w;
  }
  return true;
}

const char* reason_phrase(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    default: return "Internal Server Error";
  }
}

// ------------------------------------------------------------------ audit log
//
// kube-apiserver's --audit-log-path / --audit-policy-file for debugging test runs (the
// reference's envtest DEBUG_WRITE_AUDITLOG, odh/controllers/suite_test.go:125-137); the
// policy subset and event shape match apiserver/audit.py.  One JSON line per request at
// ResponseComplete (watches: ResponseStarted), written under a mutex.

struct Audit {
  bool on = false;
  std::string path;
  Value rules = Value::array();
  std::set<std::string> omit;
  std::mutex mu;
  std::atomic<uint64_t> events{0};
} g_audit;

struct AuditCtx {
  bool on = false;
  std::string level, verb, group, version, resource, ns, name, sub, received;
  int code = 0;
  std::string resp;  // response body (RequestResponse only)
};
thread_local AuditCtx t_aud;

bool audit_list_has(const Value* v, const std::string& x) {
  if (!v || !v->is_arr()) return true;  // unset: matches everything
  for (auto& e : v->arr)
    if (e.s == x) return true;
  return false;
}

std::string audit_level(const std::string& user, const std::string& verb, const std::string& ns,
                        const std::string& group, const std::string& resource, const std::string& sub) {
  for (auto& r : g_audit.rules.arr) {
    if (const Value* u = r.get("users"); u && u->is_arr() && !u->arr.empty() && !audit_list_has(u, user)) continue;
    if (const Value* v = r.get("verbs"); v && v->is_arr() && !v->arr.empty() && !audit_list_has(v, verb)) continue;
    if (const Value* n = r.get("namespaces"); n && n->is_arr() && !audit_list_has(n, ns)) continue;
    if (const Value* rs = r.get("resources"); rs && rs->is_arr() && !rs->arr.empty()) {
      bool hit = false;
      std::string full = sub.empty() ? resource : resource + "/" + sub;
      for (auto& gr : rs->arr) {
        if (gr.str_or("group") != group) continue;
        const Value* names = gr.get("resources");
        if (!names || !names->is_arr() || names->arr.empty() || audit_list_has(names, resource) ||
            audit_list_has(names, full)) {
          hit = true;
          break;
        }
      }
      if (!hit) continue;
    }
    std::string lv = r.str_or("level", "None");
    if (lv == "Metadata" || lv == "Request" || lv == "RequestResponse") return lv;
    return "None";
  }
  return "None";
}

std::string micro_now() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  struct tm tm;
  gmtime_r(&ts.tv_sec, &tm);
  char buf[48];
  size_t n = strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%S", &tm);
  snprintf(buf + n, sizeof(buf) - n, ".%06ldZ", ts.tv_nsec / 1000);
  return buf;
}

void audit_write(const AuditCtx& a, const std::string& uri, const std::string& ua, const std::string& req_body,
                 const char* stage) {
  if (g_audit.omit.count(stage)) return;
  Value ev = Value::object();
  ev["kind"] = Value::str("Event");
  ev["apiVersion"] = Value::str("audit.k8s.io/v1");
  ev["level"] = Value::str(a.level);
  ev["auditID"] = Value::str(uuid4());
  ev["stage"] = Value::str(stage);
  ev["requestURI"] = Value::str(uri);
  ev["verb"] = Value::str(a.verb);
  Value user = Value::object();
  user["username"] = Value::str("system:admin");
  Value groups = Value::array();
  groups.arr.push_back(Value::str("system:masters"));
  groups.arr.push_back(Value::str("system:authenticated"));
  user["groups"] = std::move(groups);
  ev["user"] = std::move(user);
  Value ips = Value::array();
  ips.arr.push_back(Value::str("127.0.0.1"));
  ev["sourceIPs"] = std::move(ips);
  ev["userAgent"] = Value::str(ua);
  Value ref = Value::object();
  ref["resource"] = Value::str(a.resource);
  if (!a.ns.empty()) ref["namespace"] = Value::str(a.ns);
  if (!a.name.empty()) ref["name"] = Value::str(a.name);
  ref["apiGroup"] = Value::str(a.group);
  ref["apiVersion"] = Value::str(a.version);
  if (!a.sub.empty()) ref["subresource"] = Value::str(a.sub);
  ev["objectRef"] = std::move(ref);
  Value rs = Value::object();
  rs["metadata"] = Value::object();
  rs["code"] = Value::integer(a.code);
  ev["responseStatus"] = std::move(rs);
  if ((a.level == "Request" || a.level == "RequestResponse") && !req_body.empty()) {
    try {
      ev["requestObject"] = kj::parse(req_body);
    } catch (const kj::ParseError&) {
    }
  }
  if (a.level == "RequestResponse" && !a.resp.empty() && std::string(stage) == "ResponseComplete") {
    try {
      ev["responseObject"] = kj::parse(a.resp);
    } catch (const kj::ParseError&) {
    }
  }
  ev["requestReceivedTimestamp"] = Value::str(a.received);
  ev["stageTimestamp"] = Value::str(micro_now());
  std::string line = kj::dump(ev) + "\n";
  std::lock_guard<std::mutex> g(g_audit.mu);
  if (FILE* f = fopen(g_audit.path.c_str(), "a")) {
    fwrite(line.data(), 1, line.size(), f);
    fclose(f);
    g_audit.events++;
  }
}

bool respond(int fd, int code, const std::string& body, bool keep_alive) {
  if (t_aud.on) {
    t_aud.code = code;
    if (t_aud.level == "RequestResponse") t_aud.resp = body;
    if (t_aud.name.empty() && t_aud.verb == "create" && code < 300) {
      // kube-apiserver names the created object in objectRef (generateName included)
      try {
        Value o = kj::parse(body);
        if (const Value* md = o.get("metadata")) t_aud.name = md->str_or("name");
      } catch (const kj::ParseError&) {
      }
    }
  }
  std::string h = "HTTP/1.1 " + std::to_string(code) + " " + reason_phrase(code) +
                  "\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) +
                  (keep_alive ? "\r\n\r\n" : "\r\nConnection: close\r\n\r\n");
  h += body;
  return write_all(fd, h.data(), h.size());
}

struct Request {
  std::string method, path, query, body, ctype, auth, user_agent, target;
  bool keep_alive = true;
  std::map<std::string, std::string> q;
};

bool read_request(Conn& c, Request& rq) {
  char tmp[65536];
  size_t hdr_end;
  while ((hdr_end = c.buf.find("\r\n\r\n")) == std::string::npos) {
    ssize_t n = recv(c.fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return false;
    c.buf.append(tmp, n);
    if (c.buf.size() > (64u << 20)) return false;
  }
  std::string head = c.buf.substr(0, hdr_end);
  c.buf.erase(0, hdr_end + 4);
  std::istringstream hs(head);
  std::string line;
  std::getline(hs, line);
  if (!line.empty() && line.back() == '\r') line.pop_back();
  std::istringstream ls(line);
  std::string target, proto;
  ls >> rq.method >> target >> proto;
  rq.target = target;
  size_t qm = target.find('?');
  rq.path = url_decode(target.substr(0, qm));
  rq.query = qm == std::string::npos ? "" : target.substr(qm + 1);
  for (auto& kv : split(rq.query, '&')) {
    if (kv.empty()) continue;
    size_t e = kv.find('=');
    rq.q[url_decode(kv.substr(0, e))] = e == std::string::npos ? "" : url_decode(kv.substr(e + 1));
  }
  size_t clen = 0;
  bool chunked = false;
  rq.keep_alive = proto != "HTTP/1.0";
  while (std::getline(hs, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string k = line.substr(0, colon), v = trim(line.substr(colon + 1));
    std::transform(k.begin(), k.end(), k.begin(), ::tolower);
    if (k == "content-length") {
      // digits only: a malformed length ends the connection instead of throwing out of the
      // connection thread (which would terminate the server)
      if (v.empty() || v.size() > 12 || v.find_first_not_of("0123456789") != std::string::npos) return false;
      clen = std::stoul(v);
    }
    else if (k == "content-type") rq.ctype = v.substr(0, v.find(';'));
    else if (k == "authorization") rq.auth = v;
    else if (k == "user-agent") rq.user_agent = v;
    else if (k == "transfer-encoding" && v.find("chunked") != std::string::npos) chunked = true;
    else if (k == "connection") {
      std::string lv = v;
      std::transform(lv.begin(), lv.end(), lv.begin(), ::tolower);
      if (lv == "close") rq.keep_alive = false;
    }
  }
  if (chunked) {
    std::string out;
    while (true) {
      size_t le;
      while ((le = c.buf.find("\r\n")) == std::string::npos) {
        ssize_t n = recv(c.fd, tmp, sizeof(tmp), 0);
        if (n <= 0) return false;
        c.buf.append(tmp, n);
      }
      std::string hex = c.buf.substr(0, c.buf.find_first_of(";\r"));
      if (hex.empty() || hex.size() > 12 || hex.find_first_not_of("0123456789abcdefABCDEF") != std::string::npos)
        return false;
      size_t sz = std::stoul(hex, nullptr, 16);
      c.buf.erase(0, le + 2);
      while (c.buf.size() < sz + 2) {
        ssize_t n = recv(c.fd, tmp, sizeof(tmp), 0);
        if (n <= 0) return false;
        c.buf.append(tmp, n);
      }
      if (sz == 0) {
        c.buf.erase(0, 2);
        break;
      }
      out.append(c.buf, 0, sz);
      c.buf.erase(0, sz + 2);
    }
    rq.body = out;
  } else {
    while (c.buf.size() < clen) {
      ssize_t n = recv(c.fd, tmp, sizeof(tmp), 0);
      if (n <= 0) return false;
      c.buf.append(tmp, n);
    }
    rq.body = c.buf.substr(0, clen);
    c.buf.erase(0, clen);
  }
  return true;
}

struct Path {
  Res* res = nullptr;
  std::string version, ns, name, sub;
};

bool parse_path(const std::string& p, Path& out) {
  std::vector<std::string> segs;
  for (auto& s : split(p, '/'))
    if (!s.empty()) segs.push_back(s);
  std::string group;
  size_t rest;
  if (segs.size() >= 3 && segs[0] == "api") {
    out.version = segs[1];
    rest = 2;
  } else if (segs.size() >= 4 && segs[0] == "apis") {
    group = segs[1];
    out.version = segs[2];
    rest = 3;
  } else {
    return false;
  }
  std::vector<std::string> r(segs.begin() + rest, segs.end());
  if (r.size() >= 3 && r[0] == "namespaces" && by_plural(group, r[2])) {
    out.ns = r[1];
    r.erase(r.begin(), r.begin() + 2);
  }
  out.res = by_plural(group, r[0]);
  if (!out.res || r.size() > 3) return false;
  if (r.size() > 1) out.name = r[1];
  if (r.size() > 2) out.sub = r[2];
  return true;
}

Value discovery(const std::string& p, bool* found) {
  *found = true;
  std::string path = p;
  while (path.size() > 1 && path.back() == '/') path.pop_back();
  if (path == "/api") {
    Value v = Value::object();
    v["kind"] = Value::str("APIVersions");
    Value vs = Value::array();
    vs.arr.push_back(Value::str("v1"));
    v["versions"] = vs;
    return v;
  }
  if (path == "/apis") {
    Value v = Value::object();
    v["kind"] = Value::str("APIGroupList");
    v["apiVersion"] = Value::str("v1");
    std::map<std::string, std::vector<std::string>> groups;
    for (auto& r : g_res)
      if (!r->group.empty() && r->installed)
        for (auto& ver : r->versions) {
          auto& l = groups[r->group];
          if (std::find(l.begin(), l.end(), ver) == l.end()) l.push_back(ver);
        }
    Value gl = Value::array();
    for (auto& kv : groups) {
      Value g = Value::object();
      g["name"] = Value::str(kv.first);
      Value vers = Value::array();
      for (auto& ver : kv.second) {
        Value x = Value::object();
        x["groupVersion"] = Value::str(kv.first + "/" + ver);
        x["version"] = Value::str(ver);
        vers.arr.push_back(x);
      }
      g["versions"] = vers;
      g["preferredVersion"] = vers.arr[0];
      gl.arr.push_back(g);
    }
    v["groups"] = gl;
    return v;
  }
  auto segs = split(path, '/');
  std::vector<std::string> s;
  for (auto& x : segs)
    if (!x.empty()) s.push_back(x);
  std::string group, version;
  if (s.size() == 2 && s[0] == "api") version = s[1];
  else if (s.size() == 3 && s[0] == "apis") {
    group = s[1];
    version = s[2];
  } else {
    *found = false;
    return Value();
  }
  Value list = Value::array();
  for (auto& r : g_res) {
    if (r->group != group || !r->installed || std::find(r->versions.begin(), r->versions.end(), version) == r->versions.end())
      continue;
    Value e = Value::object();
    e["name"] = Value::str(r->plural);
    e["singularName"] = Value::str(r->singular);
    e["namespaced"] = Value::boolean(r->namespaced);
    e["kind"] = Value::str(r->kind);
    Value verbs = Value::array();
    for (const char* vb : {"create", "delete", "get", "list", "patch", "update", "watch"}) verbs.arr.push_back(Value::str(vb));
    e["verbs"] = verbs;
    list.arr.push_back(e);
    if (r->status) {
      Value st = Value::object();
      st["name"] = Value::str(r->plural + "/status");
      st["singularName"] = Value::str("");
      st["namespaced"] = Value::boolean(r->namespaced);
      st["kind"] = Value::str(r->kind);
      list.arr.push_back(st);
    }
  }
  if (list.arr.empty()) {
    *found = false;
    return Value();
  }
  Value v = Value::object();
  v["kind"] = Value::str("APIResourceList");
  v["apiVersion"] = Value::str("v1");
  v["groupVersion"] = Value::str(group.empty() ? version : group + "/" + version);
  v["resources"] = list;
  return v;
}

bool socket_closed(int fd) {
  struct pollfd p {fd, POLLIN | POLLRDHUP, 0};
  if (poll(&p, 1, 0) > 0) {
    if (p.revents & (POLLRDHUP | POLLHUP | POLLERR)) return true;
    char c;
    ssize_t n = recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    if (n == 0) return true;
  }
  return false;
}

bool write_chunk(int fd, const std::string& data) {
  char hdr[32];
  int h = snprintf(hdr, sizeof(hdr), "%zx\r\n", data.size());
  std::string out(hdr, h);
  out += data;
  out += "\r\n";
  return write_all(fd, out.data(), out.size());
}

std::string event_line(const Res& r, const Ev& e, const std::string& version) {
  auto& c = *e.cache;
  std::lock_guard<std::mutex> g(c.mu);
  if (c.line && c.version == version) return *c.line;
  Value ev = Value::object();
  ev["type"] = Value::str(e.type);
  ev["object"] = out_obj(r, *e.obj, version);
  auto s = std::make_shared<std::string>(kj::dump(ev));
  *s += '\n';
  if (!c.line) {
    c.line = s;
    c.version = version;
  }
  return *s;
}

void serve_watch(int fd, Res& r, const Path& p, const Request& rq) {
  std::string rv = rq.q.count("resourceVersion") ? rq.q.at("resourceVersion") : "";
  if (!rv.empty() && (rv.size() > 18 || rv.find_first_not_of("0123456789") != std::string::npos)) {
    respond(fd, 400, kj::dump(status_obj(BadRequest("invalid resourceVersion " + rv))), false);
    return;
  }
  double timeout = rq.q.count("timeoutSeconds") ? std::atof(rq.q.at("timeoutSeconds").c_str()) : 1800.0;
  bool bookmarks = rq.q.count("allowWatchBookmarks") && (rq.q.at("allowWatchBookmarks") == "true" || rq.q.at("allowWatchBookmarks") == "1");
  auto lr = parse_labels(rq.q.count("labelSelector") ? rq.q.at("labelSelector") : "");
  auto fr = parse_fields(rq.q.count("fieldSelector") ? rq.q.at("fieldSelector") : "");
  std::string ns = r.namespaced ? p.ns : "";
  // by value: the slot (and this filter) may outlive the stream in a writer's queued wake-up
  auto wants = [ns, lr, fr](const Value& o) {
    if (!ns.empty() && mget(o, "namespace") != ns) return false;
    if (!lr.empty() && !match_labels(lr, o)) return false;
    if (!fr.empty() && !match_fields(fr, o)) return false;
    return true;
  };
  std::string head = "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n";
  if (!write_all(fd, head.data(), head.size())) return;
  int64_t last_seq;
  std::vector<std::string> pending;
  // shared: a writer thread may still hold it (queued wake-up) after this stream ends
  auto slot_ptr = std::make_shared<WatchSlot>();
  WatchSlot& slot = *slot_ptr;
  Bucket* wb = nullptr;
  Hist* wh = nullptr;  // the history this watch reads: its namespace's, or the kind's
  struct Unregister {  // every exit path drops the slot from the bucket's watcher index
    Bucket*& b;
    const std::string& ns;
    WatchSlot* s;
    ~Unregister() {
      if (!b) return;
      std::lock_guard<std::mutex> hg(b->hmu);
      auto rg = b->watchers.equal_range(ns);
      for (auto it = rg.first; it != rg.second; ++it)
        if (it->second.get() == s) {
          b->watchers.erase(it);
          break;
        }
    }
  } unregister{wb, ns, &slot};
  slot.wants = wants;
  slot.filtered = !lr.empty() || !fr.empty();
  {
    Bucket& b = bucket(r);
    StoreLock g(b);
    std::lock_guard<std::mutex> hg(b.hmu);
    wb = &b;
    wh = ns.empty() ? &b.all : &b.by_ns[ns];
    b.watchers.emplace(ns, slot_ptr);
    last_seq = wh->seq;
    slot.hist = wh;
    slot.seen = last_seq;
    if (rv.empty() || rv == "0") {
      for (auto& kv : b.objs)
        if (wants(*kv.second)) {
          Value ev = Value::object();
          ev["type"] = Value::str("ADDED");
          ev["object"] = out_obj(r, *kv.second, p.version);
          pending.push_back(kj::dump(ev) + "\n");
        }
    } else {
      int64_t since = std::stoll(rv);
      const std::deque<Ev>& hist = wh->hist;
      // 410 when an event after `since` has fallen off the resource's bounded history
      if (since < b.dropped_rv) {
        P.watch_gone++;
        Value ev = Value::object();
        ev["type"] = Value::str("ERROR");
        ev["object"] = status_obj(Gone());
        pending.push_back(kj::dump(ev) + "\n");
        last_seq = -1;
      } else {
        for (auto& e : hist)
          if (e.rv > since && (wants(*e.obj) || (e.old && wants(*e.old)))) pending.push_back(event_line(r, e, p.version));
      }
    }
  }
  for (auto& l : pending)
    if (!write_chunk(fd, l)) return;
  if (last_seq < 0) {
    write_all(fd, "0\r\n\r\n", 5);
    return;
  }
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds((int64_t)(timeout * 1000));
  auto last_write = std::chrono::steady_clock::now();
  uint64_t cpu_mark = thread_cpu_ns();
  while (!g_stop) {
    {  // watch CPU is booked as it accrues (a stream lives for minutes)
      uint64_t now_cpu = thread_cpu_ns();
      P.cpu_ns[C_WATCH] += now_cpu - cpu_mark;
      cpu_mark = now_cpu;
    }
    std::vector<std::string> lines;
    uint64_t oldest_ns = 0;
    bool gone = false;
    {
      Bucket& b = *wb;  // element references of S.data stay valid; buckets are never erased
      Hist& h = *wh;
      std::unique_lock<std::mutex> lk(b.hmu);
      // system_clock deadline: libstdc++ maps a steady_clock wait to pthread_cond_clockwait,
      // which ThreadSanitizer (GCC 11) does not intercept.  The timeout only paces the stream's
      // own checks (client gone; the watch deadline and the next bookmark cap it): catch-up
      // scans of a filtered watcher are emit()'s periodic wake-ups.  At 500 ms, thousands of per-namespace watch
      // threads waking twice a second were a third of the server's watch CPU at 64 namespaces
      // per rank; a wall-clock jump is harmless here
      auto nap = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
      if (bookmarks)
        nap = std::min(nap, std::chrono::duration_cast<std::chrono::milliseconds>(
                                last_write + std::chrono::seconds(10) - std::chrono::steady_clock::now()));
      nap = std::max(std::chrono::milliseconds(1), std::min(nap, std::chrono::milliseconds(5000)));
      slot.cv.wait_until(lk, std::chrono::system_clock::now() + nap,
                         [&] { return h.seq > last_seq || g_stop.load(); });
      if (h.seq > last_seq) {
        if (!h.hist.empty() && h.hist.front().seq > last_seq + 1) {
          gone = true;  // the watcher fell behind the bounded history
        } else {
          size_t start = h.hist.size() - (size_t)(h.seq - last_seq);
          P.wakeups++;
          P.scanned += h.hist.size() - start;
          // serialise outside the store lock (copy the shared event refs first)
          std::vector<Ev> evs;
          for (size_t n = start; n < h.hist.size(); ++n) {
            const Ev& e = h.hist[n];
            if (wants(*e.obj) || (e.old && wants(*e.old))) {
              evs.push_back(e);
              if (e.t_ns && (!oldest_ns || e.t_ns < oldest_ns)) oldest_ns = e.t_ns;
            }
          }
          last_seq = h.seq;
          slot.seen = last_seq;
          lk.unlock();
          for (auto& e : evs) lines.push_back(event_line(r, e, p.version));
        }
      }
    }
    if (gone) {
      P.watch_gone++;
      Value ev = Value::object();
      ev["type"] = Value::str("ERROR");
      ev["object"] = status_obj(Gone());
      write_chunk(fd, kj::dump(ev) + "\n");
      break;
    }
    if (!lines.empty()) {
      std::string batch;
      for (auto& l : lines) batch += l;
      if (!write_chunk(fd, batch)) return;
      last_write = std::chrono::steady_clock::now();
      if (g_stall_ms > 0 && oldest_ns) {  // commit -> written to this watcher's socket
        const double ms = (double)(mono_ns() - oldest_ns) / 1e6;
        if (ms >= g_stall_ms) {
          timespec ts;
          clock_gettime(CLOCK_REALTIME, &ts);
          fprintf(stderr, "stall-watchdog: watch delivery %.1f ms (%s ns=%s, %zu events) ending at %.6f\n", ms,
                  r.plural.c_str(), ns.c_str(), lines.size(), (double)ts.tv_sec + ts.tv_nsec / 1e9);
        }
      }
    }
    auto now = std::chrono::steady_clock::now();
    if (now >= deadline) break;
    if (socket_closed(fd)) return;
    if (bookmarks && now - last_write > std::chrono::seconds(10)) {
      Value bm = Value::object();
      bm["kind"] = Value::str(r.kind);
      bm["apiVersion"] = Value::str(r.api_version(p.version));
      Value m = Value::object();
      {
        StoreLock g(*wb);  // no commit of this resource in flight: every event below it was sent
        m["resourceVersion"] = Value::str(std::to_string(S.rv.load()));
      }
      bm["metadata"] = m;
      Value ev = Value::object();
      ev["type"] = Value::str("BOOKMARK");
      ev["object"] = bm;
      if (!write_chunk(fd, kj::dump(ev) + "\n")) return;
      last_write = now;
    }
  }
  write_all(fd, "0\r\n\r\n", 5);
}

bool handle(int fd, Request& rq) {
  S.requests++;
  if (!g_token.empty() && rq.auth != "Bearer " + g_token) {
    return respond(fd, 401, kj::dump(status_obj({401, "Unauthorized", "Unauthorized", Value()})), rq.keep_alive);
  }
  if (rq.method == "GET" && (rq.path == "/healthz" || rq.path == "/readyz" || rq.path == "/livez")) {
    std::string h = "HTTP/1.1 200 OK\r\nContent-Type: text/plain\r\nContent-Length: 2\r\n\r\nok";
    return write_all(fd, h.data(), h.size());
  }
  if (rq.method == "POST" && rq.path == "/debug/patch") {
    // the patch engines on their own (tests/test_patch_parity.py: property tests against
    // utils/jsonpatch.py): {"type": json|merge|strategic, "doc": …, "patch": …}
    try {
      Value in = kj::parse(rq.body);
      std::string pt = in.str_or("type");
      const Value* doc = in.get("doc");
      const Value* patch = in.get("patch");
      if (!doc || !patch) throw PatchErr{"doc and patch required"};
      Value out = Value::object();
      if (pt == "json") out["result"] = apply_json_patch(*doc, *patch);
      else if (pt == "merge") out["result"] = merge_patch(*doc, *patch);
      else if (pt == "strategic") out["result"] = strategic_patch(*doc, *patch);
      else throw PatchErr{"unknown patch type " + pt};
      return respond(fd, 200, kj::dump(out), rq.keep_alive);
    } catch (const PatchErr& e) {
      Value out = Value::object();
      out["error"] = Value::str(e.msg);
      return respond(fd, 422, kj::dump(out), rq.keep_alive);
    } catch (const kj::ParseError&) {
      return respond(fd, 400, "{\"error\":\"bad json\"}", rq.keep_alive);
    } catch (const std::exception& e) {
      return respond(fd, 500, kj::dump(status_obj(Internal(e.what()))), rq.keep_alive);
    }
  }
  if (rq.method == "POST" && rq.path == "/debug/storage-latency") {
    // the etcd-like write latency, changed while serving: {"ms": 2} (a benchmark's realistic-
    // storage block after its zero-latency window)
    try {
      Value in = kj::parse(rq.body);
      const Value* ms = in.get("ms");
      double v = -1;
      if (ms && ms->t == kj::T::Int) v = (double)ms->i;
      else if (ms && ms->t == kj::T::Double) v = ms->d;
      if (!(v >= 0 && v <= 10000)) throw PatchErr{"ms: 0..10000 required"};
      S.write_latency_us.store((int64_t)(v * 1000.0));
      return respond(fd, 200, "{\"write_latency_us\":" + std::to_string(S.write_latency_us.load()) + "}",
                     rq.keep_alive);
    } catch (const PatchErr& e) {
      return respond(fd, 400, "{\"error\":\"" + e.msg + "\"}", rq.keep_alive);
    } catch (const kj::ParseError&) {
      return respond(fd, 400, "{\"error\":\"bad json\"}", rq.keep_alive);
    }
  }
  if (rq.method == "GET" && rq.path == "/version") {
    return respond(fd, 200, "{\"major\":\"1\",\"minor\":\"32\",\"gitVersion\":\"v1.32.8-odh-kubeflow-amd-native\"}",
                   rq.keep_alive);
  }
  if (rq.method == "GET" && rq.path == "/debug/admissions") {
    uint64_t end = g_admit.seq.load();
    uint64_t from = rq.q.count("from") ? std::stoull("0" + rq.q.at("from")) : 0;
    if (end > kAdmitRing && from < end - kAdmitRing) from = end - kAdmitRing;
    std::string out = "{\"seq\":" + std::to_string(end) + ",\"us\":[";
    for (uint64_t i = from; i < end; ++i) {
      if (i != from) out += ',';
      out += std::to_string(g_admit.us[i & (kAdmitRing - 1)].load());
    }
    out += "]}";
    return respond(fd, 200, out, rq.keep_alive);
  }
  if (rq.method == "GET" && rq.path == "/metrics") {
    int64_t rv = S.rv.load();
    char buf[1024];  // the longest line below: 14 counters of up to 20 digits and their names
    snprintf(buf, sizeof(buf),
             "{\"requests\":%llu,\"writes\":%llu,\"webhook_calls\":%llu,\"resourceVersion\":%lld,\"prof\":{",
             (unsigned long long)S.requests.load(), (unsigned long long)S.writes.load(),
             (unsigned long long)S.webhook_calls.load(), (long long)rv);
    std::string out = buf;
    for (int c = 0; c < C_N; ++c) {
      snprintf(buf, sizeof(buf), "\"%s_cpu_ns\":%llu,\"%s_calls\":%llu,\"%s_lock_hold_ns\":%llu,", CAT_NAMES[c],
               (unsigned long long)P.cpu_ns[c].load(), CAT_NAMES[c], (unsigned long long)P.calls[c].load(),
               CAT_NAMES[c], (unsigned long long)P.lock_hold_ns[c].load());
      out += buf;
    }
    snprintf(buf, sizeof(buf),
             "\"lock_wait_ns\":%llu,\"lock_contended\":%llu,\"watch_wakeups\":%llu,\"watch_scanned\":%llu,"
             "\"admit_wall_ns\":%llu,\"trim_ns\":%llu,\"trim_max_ns\":%llu,\"trims\":%llu,"
             "\"webhook_dials\":%llu,\"webhook_dial_ns\":%llu,\"watch_gone\":%llu,\"process_cpu_ns\":%llu}}",
             (unsigned long long)P.lock_wait_ns.load(), (unsigned long long)P.lock_contended.load(),
             (unsigned long long)P.wakeups.load(), (unsigned long long)P.scanned.load(),
             (unsigned long long)P.admit_wall_ns.load(), (unsigned long long)P.trim_ns.load(),
             (unsigned long long)P.trim_max_ns.load(), (unsigned long long)P.trims.load(),
             (unsigned long long)P.webhook_dials.load(), (unsigned long long)P.webhook_dial_ns.load(),
             (unsigned long long)P.watch_gone.load(), (unsigned long long)process_cpu_ns());
    out += buf;
    out.pop_back();
    out += ",\"phases\":{";
    for (int i = 0; i < PH_N; ++i) {
      snprintf(buf, sizeof(buf), "%s\"%s_cpu_ns\":%llu", i ? "," : "", PHASE_NAMES[i],
               (unsigned long long)g_phase_ns[i].load());
      out += buf;
    }
    out += "}}";
    // per resource: the contended acquisitions of its store lock
    out.pop_back();
    out += ",\"locks\":{";
    bool first = true;
    for (auto& kv : S.data) {
      if (!kv.second.contended.load()) continue;
      snprintf(buf, sizeof(buf), "%s\"%s\":{\"wait_ns\":%llu,\"contended\":%llu}", first ? "" : ",",
               kv.first.c_str(), (unsigned long long)kv.second.wait_ns.load(),
               (unsigned long long)kv.second.contended.load());
      out += buf;
      first = false;
    }
    out += "}}";
    return respond(fd, 200, out, rq.keep_alive);
  }
  try {
    if (rq.method == "GET") {
      bool found;
      Value d = discovery(rq.path, &found);
      if (found) return respond(fd, 200, kj::dump(d), rq.keep_alive);
    }
    Path p;
    if (!parse_path(rq.path, p)) throw NotFound("path", rq.path);
    Res& r = res_checked(p.res);
    if (std::find(r.versions.begin(), r.versions.end(), p.version) == r.versions.end())
      throw NotFound(r.plural, "version " + p.version);
    if (!p.sub.empty() && p.sub != "status") throw NotFound(r.plural, p.name + "/" + p.sub);
    if (!r.namespaced && !p.ns.empty()) throw BadRequest(r.plural + " is not namespaced");
    auto qget = [&](const char* k) { return rq.q.count(k) ? rq.q.at(k) : std::string(); };
    if (g_audit.on) {
      std::string w = qget("watch");
      bool watch = rq.method == "GET" && p.name.empty() && (w == "1" || w == "true" || w == "True");
      std::string verb = rq.method == "GET" ? (watch ? "watch" : (p.name.empty() ? "list" : "get"))
                         : rq.method == "POST" ? "create" : rq.method == "PUT" ? "update"
                         : rq.method == "PATCH" ? "patch" : rq.method == "DELETE" ? (p.name.empty() ? "deletecollection" : "delete")
                         : rq.method;
      std::string lv = audit_level("system:admin", verb, p.ns, r.group, r.plural, p.sub);
      if (lv != "None") {
        t_aud.on = true;
        t_aud.level = lv;
        t_aud.verb = verb;
        t_aud.group = r.group;
        t_aud.version = p.version;
        t_aud.resource = r.plural;
        t_aud.ns = p.ns;
        t_aud.name = p.name;
        t_aud.sub = p.sub;
        t_aud.received = micro_now();
        t_aud.code = 200;
        t_aud.resp.clear();
        if (watch) {  // a stream: logged when it starts
          audit_write(t_aud, rq.target, rq.user_agent, "", "ResponseStarted");
          t_aud.on = false;
        }
      }
    }
    if (rq.method == "GET" && p.name.empty()) {
      std::string w = qget("watch");
      if (w == "1" || w == "true" || w == "True") {
        t_cat = C_WATCH;
        P.calls[C_WATCH]++;
        serve_watch(fd, r, p, rq);
        return false;  // watch streams end the connection
      }
      t_cat = C_LIST;
      auto lst = do_list(r, p.ns, qget("labelSelector"), qget("fieldSelector"));
      std::string body = "{\"kind\":\"" + r.list_kind + "\",\"apiVersion\":\"" + r.api_version(p.version) +
                         "\",\"metadata\":{\"resourceVersion\":\"" + std::to_string(lst.second) + "\"},\"items\":[";
      for (size_t n = 0; n < lst.first.size(); ++n) {
        if (n) body += ',';
        if (p.version == r.storage) kj::dump(body, *lst.first[n]);
        else kj::dump(body, out_obj(r, *lst.first[n], p.version));
      }
      body += "]}";
      return respond(fd, 200, body, rq.keep_alive);
    }
    if (rq.method == "GET") {
      t_cat = C_GET;
      Obj o = do_get(r, p.ns, p.name);
      return respond(fd, 200, dump_out(r, *o, p.version), rq.keep_alive);
    }
    Value body;
    if (!rq.body.empty()) {
      try {
        PhaseTimer pt(PH_PARSE);
        body = kj::parse(rq.body);
      } catch (const kj::ParseError& e) {
        throw BadRequest(std::string("invalid JSON body: ") + e.what());
      }
    }
    if (rq.method == "POST" && p.name.empty()) {
      t_cat = C_CREATE;
      if (!body.is_obj()) throw BadRequest("object body required");
      if (!body.get("kind")) body["kind"] = Value::str(r.kind);
      Obj out = do_create(r, p.ns, std::move(body), qget("dryRun") == "All");
      return respond(fd, 201, dump_out(r, *out, p.version), rq.keep_alive);
    }
    if (rq.method == "PUT" && !p.name.empty()) {
      t_cat = C_UPDATE;
      if (!body.is_obj()) throw BadRequest("object body required");
      Value& m = mdm(body);
      if (!m.str_or("name").empty() && m.str_or("name") != p.name)
        throw BadRequest("the name of the object does not match the name on the URL");
      m["name"] = Value::str(p.name);
      Obj out = do_update(r, p.ns, p.name, std::move(body), p.sub);
      return respond(fd, 200, dump_out(r, *out, p.version), rq.keep_alive);
    }
    if (rq.method == "PATCH" && !p.name.empty()) {
      t_cat = C_PATCH;
      std::string pt;
      if (rq.ctype == "application/merge-patch+json" || rq.ctype == "application/apply-patch+yaml") pt = "merge";
      else if (rq.ctype == "application/json-patch+json") pt = "json";
      else if (rq.ctype == "application/strategic-merge-patch+json") pt = "strategic";
      else
        return respond(fd, 415, kj::dump(status_obj({415, "UnsupportedMediaType", "unsupported patch type " + rq.ctype, Value()})),
                       rq.keep_alive);
      Obj out = do_patch(r, p.ns, p.name, body, pt, p.sub);
      return respond(fd, 200, dump_out(r, *out, p.version), rq.keep_alive);
    }
    if (rq.method == "DELETE" && !p.name.empty()) {
      t_cat = C_DELETE;
      Value opts = body.is_obj() ? body : Value::object();
      if (!opts.get("propagationPolicy") && !qget("propagationPolicy").empty())
        opts["propagationPolicy"] = Value::str(qget("propagationPolicy"));
      Value out = do_delete(r, p.ns, p.name, opts);
      return respond(fd, 200, kj::dump(out), rq.keep_alive);
    }
    return respond(fd, 405, kj::dump(status_obj({405, "MethodNotAllowed", rq.method + " not allowed", Value()})),
                   rq.keep_alive);
  } catch (const ApiErr& e) {
    return respond(fd, e.code, kj::dump(status_obj(e)), rq.keep_alive);
  } catch (const kj::ParseError& e) {
    return respond(fd, 400, kj::dump(status_obj(BadRequest(e.what()))), rq.keep_alive);
  } catch (const std::exception& e) {
    return respond(fd, 500, kj::dump(status_obj(Internal(e.what()))), rq.keep_alive);
  }
}

void serve_conn(int fd) {
  Conn c{fd, {}};
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  while (!g_stop) {
    Request rq;
    if (!read_request(c, rq)) break;
    t_cat = C_OTHER;
    uint64_t c0 = thread_cpu_ns();
    t_aud.on = false;
    bool more = handle(fd, rq);
    if (t_aud.on) {
      audit_write(t_aud, rq.target, rq.user_agent, rq.body, "ResponseComplete");
      t_aud.on = false;
      t_aud.resp.clear();
    }
    if (t_cat != C_WATCH) {  // a watch books its own CPU as it goes
      P.cpu_ns[t_cat] += thread_cpu_ns() - c0;
      P.calls[t_cat]++;
    }
    if (!more) break;
    if (!rq.keep_alive) break;
  }
  close(fd);
}

void load_config(const std::string& path) {
  std::ifstream f(path);
  std::stringstream ss;
  ss << f.rdbuf();
  Value cfg = kj::parse(ss.str());
  const Value* res = cfg.get("resources");
  if (!res || !res->is_arr()) throw std::runtime_error("config: resources[] required");
  for (auto& r : res->arr) {
    auto x = std::make_unique<Res>();
    x->group = r.str_or("group");
    x->kind = r.str_or("kind");
    x->plural = r.str_or("plural");
    x->singular = r.str_or("singular");
    x->list_kind = r.str_or("listKind", x->kind + "List");
    x->storage = r.str_or("storageVersion");
    x->key = x->group.empty() ? x->plural : x->plural + "." + x->group;
    if (const Value* v = r.get("versions"))
      for (auto& s : v->arr) x->versions.push_back(s.s);
    if (const Value* v = r.get("namespaced")) x->namespaced = v->b;
    if (const Value* v = r.get("status")) x->status = v->b;
    if (const Value* v = r.get("installed")) x->installed = v->b;
    g_res.push_back(std::move(x));
  }
  if (const Value* v = cfg.get("gc")) S.gc = v->b;
  if (const Value* v = cfg.get("defaulting")) S.defaulting = v->b;
  if (const Value* v = cfg.get("schemas"); v && v->is_obj())
    for (auto& m : v->obj) g_schemas[m.k] = m.v;
  if (const Value* v = cfg.get("history"))
    if (v->t == T::Int) S.history = (size_t)v->i;
  g_token = cfg.str_or("token");
  if (const Value* a = cfg.get("audit"); a && a->is_obj()) {
    g_audit.path = a->str_or("path");
    if (const Value* pol = a->get("policy"); pol && pol->is_obj()) {
      if (const Value* rules = pol->get("rules"); rules && rules->is_arr()) g_audit.rules = *rules;
      if (const Value* om = pol->get("omitStages"); om && om->is_arr())
        for (auto& x : om->arr) g_audit.omit.insert(x.s);
    }
    g_audit.on = !g_audit.path.empty();
  }
}

}  // namespace

int main(int argc, char** argv) {
  // started by the benchmark / test platform (utils/procutil.py): die with the launcher
  if (const char* parent = std::getenv("ODH_PDEATHSIG_PARENT")) {
    prctl(PR_SET_PDEATHSIG, SIGTERM);
    if (std::to_string(getppid()) != parent) raise(SIGTERM);  // it died before we armed
    unsetenv("ODH_PDEATHSIG_PARENT");
  }
  std::string host = "127.0.0.1", config;
  int port = 0;
  for (int k = 1; k < argc; ++k) {
    std::string a = argv[k];
    auto next = [&]() { return k + 1 < argc ? std::string(argv[++k]) : std::string(); };
    if (a == "--host") host = next();
    else if (a == "--port") port = std::stoi(next());
    else if (a == "--config") config = next();
    else if (a == "--gc") S.gc = true;
    else if (a == "--token") g_token = next();
    else if (a == "--history") S.history = std::stoul(next());
    else if (a == "--write-latency-ms") S.write_latency_us = (int64_t)(std::stod(next()) * 1000.0);
    else if (a == "--webhook-connections") g_webhook_conns = std::max(1, std::stoi(next()));
    else {
      fprintf(stderr, "unknown flag %s\n", a.c_str());
      return 2;
    }
  }
  if (config.empty()) {
    fprintf(stderr, "--config scheme.json is required\n");
    return 2;
  }
  bool gc_flag = S.gc;
  std::string tok = g_token;
  size_t hist = S.history;
  load_config(config);
  init_buckets();
  // One connection per thread, so glibc gives each busy thread its own malloc arena (up to
  // 8 x cores), and objects freed on one thread were often allocated on another: freed memory
  // spreads over many half-empty arenas.  A periodic trim returns it.  The arena count is left
  // at glibc's default: capping it at 8 (MALLOC_ARENA_MAX, still honoured) cut the resident
  // size by ≈10 % but cost ≈35 % more CPU per request at 4 ranks on a 64-core MI355X box, every
  // thread queueing on a shared arena lock (tools/research/apiserver_ab.sh, profiles/r4_apiab).
  // ODH_APISERVER_TRIM_S: the trim period (seconds; 0 turns the trim off — diagnostics)
  double trim_s = 2.0;
  if (const char* e = std::getenv("ODH_APISERVER_TRIM_S")) trim_s = std::atof(e);
  if (trim_s > 0)
    std::thread([trim_s] {
      while (!g_stop) {
        std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(trim_s * 1e6)));
        auto t0 = std::chrono::steady_clock::now();
        malloc_trim(0);
        uint64_t d = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        P.trim_ns += d;
        P.trims++;
        if (d > P.trim_max_ns.load()) P.trim_max_ns = d;
        if (g_stall_ms > 0 && d >= (uint64_t)g_stall_ms * 1000000ull)
          fprintf(stderr, "stall-watchdog: malloc_trim took %.1f ms\n", (double)d / 1e6);
      }
    }).detach();
  // ODH_STALL_WATCHDOG_MS (diagnostics): a thread that sleeps 1 ms and allocates a page at a
  // time reports to stderr, with the wall-clock end, every iteration that took this long —
  // a stall of the whole process (scheduling, the address-space lock, an allocator lock)
  // shows up here, a stall of one request path does not
  if (const char* e = std::getenv("ODH_STALL_WATCHDOG_MS")) g_stall_ms = std::atoi(e);
  if (g_stall_ms > 0)
    std::thread([] {
      while (!g_stop) {
        auto t0 = std::chrono::steady_clock::now();
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        void* pg = malloc(4096);
        if (pg) {
          static_cast<volatile char*>(pg)[0] = 1;
          free(pg);
        }
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms >= g_stall_ms) {
          timespec ts;
          clock_gettime(CLOCK_REALTIME, &ts);
          fprintf(stderr, "stall-watchdog: %.1f ms ending at %.6f\n", ms, (double)ts.tv_sec + ts.tv_nsec / 1e9);
        }
      }
    }).detach();
  if (gc_flag) S.gc = true;
  if (!tok.empty()) g_token = tok;
  if (hist != 512) S.history = hist;
  signal(SIGPIPE, SIG_IGN);
  SSL_library_init();
  SSL_load_error_strings();
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  struct sockaddr_in addr {};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(port);
  inet_pton(AF_INET, host.c_str(), &addr.sin_addr);
  if (bind(ls, (struct sockaddr*)&addr, sizeof(addr)) != 0) {
    perror("bind");
    return 1;
  }
  listen(ls, 1024);
  socklen_t len = sizeof(addr);
  getsockname(ls, (struct sockaddr*)&addr, &len);
  printf("LISTENING %d\n", ntohs(addr.sin_port));
  fflush(stdout);
  while (true) {
    int fd = accept(ls, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (g_stall_ms > 0) {  // diagnostics: a connection's thread slow to start delays its requests
      const uint64_t t0 = mono_ns();
      struct tcp_info ti {};
      socklen_t tl = sizeof(ti);
      // how long the connection sat in the listen queue: its handshake (and any request bytes)
      // arrived this long before accept() handed it over
      if (getsockopt(fd, IPPROTO_TCP, TCP_INFO, &ti, &tl) == 0 && ti.tcpi_last_data_recv >= (unsigned)g_stall_ms) {
        timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        fprintf(stderr, "stall-watchdog: accepted %u ms after its first data (last ack recv %u ms) at %.6f\n",
                ti.tcpi_last_data_recv, ti.tcpi_last_ack_recv, (double)ts.tv_sec + ts.tv_nsec / 1e9);
      }
      std::thread([fd, t0] {
        const double ms = (double)(mono_ns() - t0) / 1e6;
        if (ms >= g_stall_ms) {
          timespec ts;
          clock_gettime(CLOCK_REALTIME, &ts);
          fprintf(stderr, "stall-watchdog: connection thread started %.1f ms after accept, at %.6f\n", ms,
                  (double)ts.tv_sec + ts.tv_nsec / 1e9);
        }
        serve_conn(fd);
      }).detach();
      const double sp = (double)(mono_ns() - t0) / 1e6;
      if (sp >= g_stall_ms) fprintf(stderr, "stall-watchdog: thread spawn took %.1f ms\n", sp);
      continue;
    }
    std::thread(serve_conn, fd).detach();
  }
  return 0;
}
