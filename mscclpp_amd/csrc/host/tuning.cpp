// Data-driven algorithm selection for one MI355X node: a store of tuned configurations per
// (hardware profile, collective, message size), in the JSON format of the reference's tuner
// (python/mscclpp_benchmark/tuning_config.py:37-200):
//   {"version": 1, "profiles": [{"sku": "MI355X", "scale": 8,
//     "collectives": {"allreduce": [{"message_size": 16384, "algorithm": "default_allreduce_packet",
//                                    "nblocks": 56, "nthreads": 512, "time_us": 9.1}, ...]}}]}
// A profile matches when its sku (normalised like normalize_sku, tuning_config.py:101-107) and scale
// (ranks) equal the runtime's or are absent; the most specific match wins (:120-142).  Within a
// collective the entry chosen is the one with the largest message_size <= the message, or the first
// entry for a smaller message (bisect_left rule, :145-157).
//
// The built-in table restates algorithm_selector.cc:91-139 (AMD branch) as data: <= 16 KiB one-hop
// LL8, <= 1 MiB two-hop LL16, larger the bulk all-pairs path.  At 2 ranks (its own profile) one-hop
// LL8 takes the whole LL range: there both LL forms put the same bytes on the one link, and the one
// hop measured 4.0-4.2 against 5.2-5.6 us at 1-256 KiB, 4.4 / 6.2 against 7.3 / 9.5 us at 512 KiB /
// 1 MiB (profiles/r3k_inprocess_ll_probe_n2_ll8.json, r3n_inprocess_ll8_probe_n2_shapes.json,
// 2 ranks in one launch, fabric-free).  MSCCLPP_AMD_TUNED_CONFIG names a file
// whose profiles are consulted first (e.g. the `tuned_config` that bench.py prints after tuning on
// the node); mscclppAmdTunedConfigLoad does the same at run time.
#include <atomic>
#include <fstream>
#include <sstream>

#include "comm_internal.hpp"
#include "json.hpp"

namespace mscclpp_amd {
namespace host {

namespace {

struct Entry {
  uint64_t size;
  std::string algorithm;
  int nblocks = 0, nthreads = 0;
  std::string source;  // "reference", "fabric-free", "tuned" (loaded files), or the file's own tag
};
struct Profile {
  std::string sku;  // empty: any
  int scale = 0;    // 0: any
  std::map<std::string, std::vector<Entry>> byCollective;  // sorted by size
};

// Every entry says where it came from ("source"): "reference" restates the reference's selector;
// "fabric-free" was measured with all ranks on one GPU (in-process or shared-device sweeps), which
// prices the hand-off but no link bytes -- a guess for the node until a node-measured table (bench.py
// prints one as `tuned_config_table`) overrides it.  Entries of a loaded file without a source are
// "tuned".  "reference; grid fabric-free": the reference's choice of algorithm, run on the kernel's
// default grid, whose few-rank cap (max(16, 48 / (n-1)) workgroups per peer, allreduce_ll.hip) came
// from fabric-free sweeps -- an entry with nblocks / nthreads replaces it.
// mscclppAmdTunedConfigSource reports which entry applied.
const char* kBuiltin = R"({"version": 1, "profiles": [
  {"scale": 2, "collectives": {"allreduce": [
      {"message_size": 1, "algorithm": "default_allreduce_allpair_packet", "source": "fabric-free"},
      {"message_size": 1048577, "algorithm": "default_allreduce_fullmesh", "source": "reference"}]}},
  {"collectives": {
    "allreduce": [
      {"message_size": 1, "algorithm": "default_allreduce_allpair_packet", "source": "reference"},
      {"message_size": 16385, "algorithm": "default_allreduce_packet",
       "source": "reference; grid fabric-free"},
      {"message_size": 1048577, "algorithm": "default_allreduce_fullmesh", "source": "reference"}],
    "allgather": [{"message_size": 1, "algorithm": "default_allgather_fullmesh2", "source": "reference"}],
    "reducescatter": [{"message_size": 1, "algorithm": "default_reducescatter_fullmesh", "source": "reference"}]}}
]})";

std::string normalizeSku(const std::string& raw) {
  std::string up;
  for (char c : raw) up += (char)std::toupper((unsigned char)c);
  for (const char* known : {"MI355X", "MI350X", "MI325X", "MI300X", "GB300", "GB200", "H100", "A100"})
    if (up.find(known) != std::string::npos) return known;
  std::string out;
  for (char c : up) out += std::isalnum((unsigned char)c) ? c : '_';
  return out.empty() ? "UNKNOWN" : out;
}

std::vector<Profile> parseStore(const std::string& text, const char* defaultSource) {
  const json::Value doc = json::parse(text);
  if (!doc.isObject() || !doc.contains("profiles") || !doc["profiles"].isArray())
    throw std::invalid_argument("tuned config: expected an object with a 'profiles' list");
  std::vector<Profile> out;
  for (const auto& p : doc["profiles"].arr) {
    Profile prof;
    if (p.contains("sku")) prof.sku = normalizeSku(p["sku"].str());
    if (p.contains("scale")) prof.scale = (int)p["scale"].asI64();
    if (p.contains("collectives")) {
      for (const auto& kv : p["collectives"].obj) {
        const json::Value& list = kv.second.isObject() && kv.second.contains("configs") ? kv.second["configs"] : kv.second;
        if (!list.isArray()) continue;
        std::vector<Entry> es;
        for (const auto& e : list.arr) {
          Entry en;
          en.size = e["message_size"].asU64();
          if (en.size == 0) throw std::invalid_argument("tuned config: message_size must be positive");
          en.algorithm = e["algorithm"].str();
          if (e.contains("nblocks") && e["nblocks"].kind != json::Value::Null) en.nblocks = (int)e["nblocks"].asI64();
          if (e.contains("nthreads") && e["nthreads"].kind != json::Value::Null) en.nthreads = (int)e["nthreads"].asI64();
          en.source = e.contains("source") && e["source"].kind != json::Value::Null ? e["source"].str() : defaultSource;
          es.push_back(en);
        }
        std::sort(es.begin(), es.end(), [](const Entry& a, const Entry& b) { return a.size < b.size; });
        prof.byCollective[kv.first] = es;
      }
    }
    out.push_back(std::move(prof));
  }
  return out;
}

const Entry* selectIn(const std::vector<Entry>& es, uint64_t size) {
  if (es.empty()) return nullptr;
  size_t i = 0;
  while (i < es.size() && es[i].size < size) ++i;  // bisect_left
  if (i == es.size()) return &es.back();
  if (es[i].size == size || i == 0) return &es[i];
  return &es[i - 1];
}

// Bumped whenever the store's contents change, so callers that memoise a decision taken from it
// (comm.cpp's selection memo) know to take it again.
std::atomic<uint64_t> gTunedGen{1};

struct Store {
  std::mutex mu;
  std::vector<Profile> user, builtin;
  std::string sku;
  bool init = false;
};

Store& store() {
  static Store s;
  std::lock_guard<std::mutex> lk(s.mu);
  if (!s.init) {
    s.init = true;
    s.builtin = parseStore(kBuiltin, "builtin");
    int dev = 0;
    hipDeviceProp_t prop{};
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) {
      s.sku = normalizeSku(prop.name);
      if (s.sku == "UNKNOWN" || s.sku.empty()) s.sku = normalizeSku(prop.gcnArchName);
    }
    (void)hipGetLastError();
    if (const char* path = std::getenv("MSCCLPP_AMD_TUNED_CONFIG")) {
      try {
        std::ifstream f(path);
        std::stringstream ss;
        ss << f.rdbuf();
        s.user = parseStore(ss.str(), "tuned");
        gTunedGen.fetch_add(1);
      } catch (const std::exception& e) {
        warn(std::string("MSCCLPP_AMD_TUNED_CONFIG ignored: ") + e.what());
      }
    }
  }
  return s;
}

const Entry* selectProfiles(const std::vector<Profile>& ps, const std::string& sku, int scale,
                            const std::string& coll, uint64_t size) {
  int best = -1;
  const Entry* chosen = nullptr;
  for (const auto& p : ps) {
    int spec = 0;
    if (!p.sku.empty()) {
      if (p.sku != sku) continue;
      ++spec;
    }
    if (p.scale) {
      if (p.scale != scale) continue;
      ++spec;
    }
    auto it = p.byCollective.find(coll);
    if (it == p.byCollective.end()) continue;
    const Entry* e = selectIn(it->second, size);
    if (e && spec > best) {
      best = spec;
      chosen = e;
    }
  }
  return chosen;
}

}  // namespace

uint64_t tunedGeneration() {
  (void)store();  // the built-in table and MSCCLPP_AMD_TUNED_CONFIG are read on first use
  return gTunedGen.load(std::memory_order_relaxed);
}

bool tunedConfig(const std::string& collective, int nranks, uint64_t bytes, std::string& algorithm, int& nblocks,
                 int& nthreads, std::string* source) {
  Store& s = store();
  std::lock_guard<std::mutex> lk(s.mu);
  const Entry* e = selectProfiles(s.user, s.sku, nranks, collective, bytes);
  if (!e) e = selectProfiles(s.builtin, s.sku, nranks, collective, bytes);
  if (!e) return false;
  algorithm = e->algorithm;
  nblocks = e->nblocks;
  nthreads = e->nthreads;
  if (source) *source = e->source;
  return true;
}

int algoCodeOf(const std::string& name) {
  if (name == "default_allreduce_packet") return MSCCLPP_AMD_ALGO_PACKET;
  if (name == "default_allreduce_allpair_packet") return MSCCLPP_AMD_ALGO_ALLPAIR;
  if (name == "default_allreduce_fullmesh") return MSCCLPP_AMD_ALGO_FULLMESH;
  if (name == "default_allreduce_rsag") return MSCCLPP_AMD_ALGO_RSAG;
  if (name == "default_allreduce_rsag_zero_copy") return MSCCLPP_AMD_ALGO_RSAG_ZC;
  if (name == "default_allreduce_rsag_pipeline") return MSCCLPP_AMD_ALGO_RSAG_PIPELINE;
  return -1;
}

}  // namespace host
}  // namespace mscclpp_amd

extern "C" int mscclppAmdTunedConfigLoad(const char* path) {
  return guarded([&] {
    if (!path) return (int)ncclInvalidArgument;
    std::ifstream f(path);
    if (!f) return (int)ncclInvalidArgument;
    std::stringstream ss;
    ss << f.rdbuf();
    auto parsed = parseStore(ss.str(), "tuned");  // throws std::invalid_argument on a malformed file
    Store& s = store();
    std::lock_guard<std::mutex> lk(s.mu);
    s.user = std::move(parsed);
    gTunedGen.fetch_add(1);
    return (int)ncclSuccess;
  });
}

extern "C" int mscclppAmdTunedConfig(const char* collective, int nranks, size_t bytes, char* algorithm,
                                     size_t algorithmLen, int* nblocks, int* nthreads) {
  return guarded([&] {
    if (!collective) return (int)ncclInvalidArgument;
    std::string name;
    int nb = 0, nt = 0;
    if (!tunedConfig(collective, nranks, bytes, name, nb, nt)) return (int)ncclInvalidUsage;
    if (algorithm && algorithmLen) {
      std::snprintf(algorithm, algorithmLen, "%s", name.c_str());
    }
    if (nblocks) *nblocks = nb;
    if (nthreads) *nthreads = nt;
    return (int)ncclSuccess;
  });
}

extern "C" int mscclppAmdTunedConfigSource(const char* collective, int nranks, size_t bytes, char* source,
                                           size_t sourceLen) {
  return guarded([&] {
    if (!collective) return (int)ncclInvalidArgument;
    std::string name, src;
    int nb = 0, nt = 0;
    if (!tunedConfig(collective, nranks, bytes, name, nb, nt, &src)) return (int)ncclInvalidUsage;
    if (source && sourceLen) std::snprintf(source, sourceLen, "%s", src.c_str());
    return (int)ncclSuccess;
  });
}
