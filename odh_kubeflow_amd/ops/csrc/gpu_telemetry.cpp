// amdgpu busy / VRAM telemetry for the GPU-busy culler (host C++, no HIP calls).
//
// The reference culls on Jupyter kernel last-activity only
// (kf/controllers/culling_controller.go:161-196, 243-273).  On an MI355X node the
// accelerator itself is the better idleness signal, and sampling it must be cheap,
// independent of the Python GIL and never touch the GPU queues of the notebooks it
// watches.  This library therefore reads the amdgpu sysfs counters directly:
//
//   <root>/class/kfd/kfd/topology/nodes/<n>/properties   -> GPU nodes (simd_count > 0),
//        drm_render_minor, location_id (PCI BDF), unique_id (physical device id)
//   <root>/class/drm/renderD<minor>/device/gpu_busy_percent
//   <root>/class/drm/renderD<minor>/device/mem_info_vram_used | mem_info_vram_total
//
// and keeps a per-device ring of samples filled by one background thread, so the
// culler asks "mean / max busy over the last W seconds" without ever blocking on I/O.
// Partition modes (CPX/DPX) expose several KFD nodes per physical MI355X; they share
// one unique_id and one busy counter, which `physical` reports.
//
// `root` is "/sys" in production; tests point it at a synthetic tree.

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Sample {
  int64_t t_ns;
  int busy;          // percent, -1 = unavailable
  int64_t vram_used;  // bytes, -1 = unavailable
};

struct Device {
  int node = -1;           // KFD topology node id
  int render_minor = -1;
  uint64_t unique_id = 0;
  uint64_t location_id = 0;
  int domain = 0;          // PCI domain (KFD `domain` property)
  int64_t gpu_id = 0;      // KFD gpu_id: the suffix of /sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>
  int physical = -1;       // index of the first device sharing unique_id
  int64_t vram_total = -1;
  std::string dev_dir;
  std::vector<Sample> ring;
  size_t head = 0, count = 0;
  std::mutex mu;
};

struct Telemetry {
  std::string root;
  std::vector<Device*> devs;
  std::thread thr;
  std::atomic<bool> running{false};
  int interval_ms = 100;
  size_t capacity = 0;
  std::atomic<uint64_t> sweeps{0};
};

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

bool read_i64(const std::string& path, int64_t* out) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[64];
  size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  if (n == 0) return false;
  buf[n] = 0;
  char* end = nullptr;
  long long v = std::strtoll(buf, &end, 10);
  if (end == buf) return false;
  *out = (int64_t)v;
  return true;
}

void parse_properties(const std::string& path, Device* d, int64_t* simd_count) {
  std::ifstream in(path);
  std::string key;
  unsigned long long val;
  *simd_count = 0;
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    if (!(ls >> key >> val)) continue;
    if (key == "simd_count") *simd_count = (int64_t)val;
    else if (key == "drm_render_minor") d->render_minor = (int)val;
    else if (key == "unique_id") d->unique_id = val;
    else if (key == "location_id") d->location_id = val;
    else if (key == "domain") d->domain = (int)val;
  }
}

void sample_one(Device* d, Sample* s) {
  s->t_ns = now_ns();
  int64_t v;
  s->busy = read_i64(d->dev_dir + "/gpu_busy_percent", &v) ? (int)v : -1;
  s->vram_used = read_i64(d->dev_dir + "/mem_info_vram_used", &v) ? v : -1;
}

void push(Device* d, const Sample& s) {
  std::lock_guard<std::mutex> g(d->mu);
  if (d->ring.empty()) return;
  d->ring[d->head] = s;
  d->head = (d->head + 1) % d->ring.size();
  if (d->count < d->ring.size()) d->count++;
}

void sampler(Telemetry* t) {
  while (t->running.load(std::memory_order_relaxed)) {
    const auto start = std::chrono::steady_clock::now();
    for (Device* d : t->devs) {
      Sample s;
      sample_one(d, &s);
      push(d, s);
    }
    t->sweeps.fetch_add(1, std::memory_order_relaxed);
    const auto next = start + std::chrono::milliseconds(t->interval_ms);
    while (t->running.load(std::memory_order_relaxed) && std::chrono::steady_clock::now() < next)
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min(t->interval_ms, 10)));
  }
}

// Pod UID from the text of /proc/<pid>/cgroup.  The kubelet names pod cgroups after the pod
// UID, with '_' for '-' under the systemd driver:
//   v2/systemd  0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod1b2c..._9f.slice/cri-containerd-<id>.scope
//   v1/cgroupfs 12:memory:/kubepods/besteffort/pod1b2c...-9f/<id>
//   guaranteed  0::/kubepods.slice/kubepods-pod1b2c..._9f.slice/...
bool pod_uid_from_cgroup(const std::string& text, std::string* uid) {
  static const int dash_at[4] = {8, 13, 18, 23};
  for (size_t p = text.find("pod"); p != std::string::npos; p = text.find("pod", p + 1)) {
    const size_t b = p + 3;
    if (b + 36 > text.size()) break;
    bool ok = true;
    std::string u(36, '-');
    for (int i = 0; i < 36 && ok; ++i) {
      const char c = text[b + i];
      const bool sep = i == dash_at[0] || i == dash_at[1] || i == dash_at[2] || i == dash_at[3];
      if (sep) {
        ok = c == '-' || c == '_';
      } else {
        ok = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f');
        u[i] = c;
      }
    }
    if (ok) {
      *uid = u;
      return true;
    }
  }
  return false;
}

std::string read_text(const std::string& path, size_t limit = 1 << 16) {
  std::string out;
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return out;
  char buf[4096];
  size_t n;
  while (out.size() < limit && (n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
  std::fclose(f);
  return out;
}

}  // namespace

extern "C" {

struct odh_tel_info {
  int node;
  int render_minor;
  int physical;
  int domain;
  uint64_t unique_id;
  uint64_t location_id;
  int64_t vram_total;
  int64_t gpu_id;
};

struct odh_tel_sample {
  int64_t t_ns;
  int busy;
  int reserved;
  int64_t vram_used;
};

struct odh_tel_window {
  int n;
  int unavailable;  // samples whose busy counter could not be read
  double busy_mean;
  int busy_max;
  int reserved;
  double vram_used_mean;
  int64_t span_ns;
};

void* odh_tel_open(const char* root) {
  Telemetry* t = new Telemetry();
  t->root = root && *root ? root : "/sys";
  const std::string nodes = t->root + "/class/kfd/kfd/topology/nodes";
  std::vector<int> ids;
  if (DIR* dir = opendir(nodes.c_str())) {
    while (dirent* e = readdir(dir)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      ids.push_back(std::atoi(e->d_name));
    }
    closedir(dir);
  }
  std::sort(ids.begin(), ids.end());
  for (int id : ids) {
    Device* d = new Device();
    d->node = id;
    int64_t simd = 0;
    parse_properties(nodes + "/" + std::to_string(id) + "/properties", d, &simd);
    if (simd <= 0 || d->render_minor < 0) {  // CPU node
      delete d;
      continue;
    }
    d->dev_dir = t->root + "/class/drm/renderD" + std::to_string(d->render_minor) + "/device";
    int64_t v;
    if (read_i64(nodes + "/" + std::to_string(id) + "/gpu_id", &v)) d->gpu_id = v;
    d->vram_total = read_i64(d->dev_dir + "/mem_info_vram_total", &v) ? v : -1;
    d->physical = (int)t->devs.size();
    for (size_t i = 0; i < t->devs.size(); ++i)
      if (d->unique_id != 0 && t->devs[i]->unique_id == d->unique_id) {
        d->physical = t->devs[i]->physical;
        break;
      }
    t->devs.push_back(d);
  }
  return t;
}

int odh_tel_count(void* h) { return h ? (int)((Telemetry*)h)->devs.size() : 0; }

int odh_tel_info_get(void* h, int idx, odh_tel_info* out) {
  Telemetry* t = (Telemetry*)h;
  if (!t || idx < 0 || idx >= (int)t->devs.size() || !out) return -1;
  Device* d = t->devs[idx];
  out->node = d->node;
  out->render_minor = d->render_minor;
  out->physical = d->physical;
  out->domain = d->domain;
  out->unique_id = d->unique_id;
  out->location_id = d->location_id;
  out->vram_total = d->vram_total;
  out->gpu_id = d->gpu_id;
  return 0;
}

int odh_tel_read(void* h, int idx, odh_tel_sample* out) {
  Telemetry* t = (Telemetry*)h;
  if (!t || idx < 0 || idx >= (int)t->devs.size() || !out) return -1;
  Sample s;
  sample_one(t->devs[idx], &s);
  out->t_ns = s.t_ns;
  out->busy = s.busy;
  out->reserved = 0;
  out->vram_used = s.vram_used;
  return 0;
}

int odh_tel_start(void* h, int interval_ms, int capacity) {
  Telemetry* t = (Telemetry*)h;
  if (!t || interval_ms <= 0 || capacity <= 0) return -1;
  if (t->running.load()) return 0;
  t->interval_ms = interval_ms;
  t->capacity = (size_t)capacity;
  for (Device* d : t->devs) {
    std::lock_guard<std::mutex> g(d->mu);
    d->ring.assign(t->capacity, Sample{0, -1, -1});
    d->head = d->count = 0;
  }
  t->running.store(true);
  t->thr = std::thread(sampler, t);
  return 0;
}

uint64_t odh_tel_sweeps(void* h) { return h ? ((Telemetry*)h)->sweeps.load() : 0; }

// Inject a sample (tests / external samplers, e.g. amd-smi when sysfs is not mounted).
int odh_tel_push(void* h, int idx, int64_t t_ns, int busy, int64_t vram_used) {
  Telemetry* t = (Telemetry*)h;
  if (!t || idx < 0 || idx >= (int)t->devs.size()) return -1;
  Device* d = t->devs[idx];
  {
    std::lock_guard<std::mutex> g(d->mu);
    if (d->ring.empty()) d->ring.assign(t->capacity ? t->capacity : 1024, Sample{0, -1, -1});
  }
  push(d, Sample{t_ns ? t_ns : now_ns(), busy, vram_used});
  return 0;
}

int odh_tel_window_get(void* h, int idx, double seconds, odh_tel_window* out) {
  Telemetry* t = (Telemetry*)h;
  if (!t || idx < 0 || idx >= (int)t->devs.size() || !out) return -1;
  Device* d = t->devs[idx];
  std::memset(out, 0, sizeof(*out));
  out->busy_max = -1;
  const int64_t now = now_ns();
  const int64_t horizon = now - (int64_t)(seconds * 1e9);
  std::lock_guard<std::mutex> g(d->mu);
  const size_t cap = d->ring.size();
  double bsum = 0, vsum = 0;
  int nb = 0, nv = 0;
  int64_t oldest = now, newest = 0;
  for (size_t i = 0; i < d->count; ++i) {
    const Sample& s = d->ring[(d->head + cap - 1 - i) % cap];
    if (s.t_ns < horizon) break;
    out->n++;
    oldest = std::min(oldest, s.t_ns);
    newest = std::max(newest, s.t_ns);
    if (s.busy < 0) {
      out->unavailable++;
    } else {
      bsum += s.busy;
      nb++;
      out->busy_max = std::max(out->busy_max, s.busy);
    }
    if (s.vram_used >= 0) {
      vsum += (double)s.vram_used;
      nv++;
    }
  }
  out->busy_mean = nb ? bsum / nb : -1.0;
  out->vram_used_mean = nv ? vsum / nv : -1.0;
  out->span_ns = out->n ? newest - oldest : 0;
  return 0;
}

void odh_tel_stop(void* h) {
  Telemetry* t = (Telemetry*)h;
  if (!t) return;
  if (t->running.exchange(false) && t->thr.joinable()) t->thr.join();
}

void odh_tel_close(void* h) {
  Telemetry* t = (Telemetry*)h;
  if (!t) return;
  odh_tel_stop(h);
  for (Device* d : t->devs) delete d;
  delete t;
}

// Per-process GPU memory from KFD joined with the process's pod, for pod -> GPU attribution
// on a real node (no pod annotation involved):
//   <sys_root>/class/kfd/kfd/proc/<pid>/vram_<gpu_id>   bytes of VRAM the process holds on that GPU
//   <proc_root>/<pid>/cgroup                              -> pod UID (see pod_uid_from_cgroup)
// Writes one line per (pid, gpu_id) with a readable vram file: "pid gpu_id vram_bytes pod_uid\n"
// (pod_uid "-" when the process is not in a pod cgroup).  Returns the number of bytes the
// full report needs; the report is written only if it fits in `cap` (else call again).
int64_t odh_tel_kfd_procs(void* h, const char* proc_root, char* buf, int64_t cap) {
  Telemetry* t = (Telemetry*)h;
  if (!t) return -1;
  const std::string kfd = t->root + "/class/kfd/kfd/proc";
  const std::string proc = proc_root && *proc_root ? proc_root : "/proc";
  std::string report;
  DIR* dir = opendir(kfd.c_str());
  if (!dir) return 0;
  std::vector<std::string> pids;
  while (dirent* e = readdir(dir))
    if (e->d_name[0] >= '0' && e->d_name[0] <= '9') pids.emplace_back(e->d_name);
  closedir(dir);
  std::sort(pids.begin(), pids.end());
  for (const std::string& pid : pids) {
    const std::string pdir = kfd + "/" + pid;
    DIR* pd = opendir(pdir.c_str());
    if (!pd) continue;  // the process exited between the two readdirs
    std::string uid;
    bool have_uid = false, looked = false;
    while (dirent* e = readdir(pd)) {
      if (std::strncmp(e->d_name, "vram_", 5) != 0) continue;
      int64_t bytes;
      if (!read_i64(pdir + "/" + e->d_name, &bytes)) continue;
      if (!looked) {
        have_uid = pod_uid_from_cgroup(read_text(proc + "/" + pid + "/cgroup"), &uid);
        looked = true;
      }
      report += pid + " " + (e->d_name + 5) + " " + std::to_string(bytes) + " " + (have_uid ? uid : "-") + "\n";
    }
    closedir(pd);
  }
  if ((int64_t)report.size() <= cap && buf) std::memcpy(buf, report.data(), report.size());
  return (int64_t)report.size();
}

}  // extern "C"
