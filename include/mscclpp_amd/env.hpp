// The reference's environment snapshot with its spellings (include/mscclpp/env.hpp,
// src/core/env.cpp:15-70): mscclpp::env() returns one process-wide Env whose fields hold the
// MSCCLPP_* variables as set at first use (strings verbatim, booleans true unless "0", integers by
// atoi), with the reference's defaults.  What this build acts on: MSCCLPP_LOG_LEVEL,
// MSCCLPP_NCCL_LIB_PATH and MSCCLPP_FORCE_NCCL_FALLBACK_OPERATION (the vendor fallback),
// MSCCLPP_NCCL_SYMMETRIC_MEMORY; its own knobs are MSCCLPP_AMD_* (INTEGRATION.md).  The InfiniBand,
// NVLS and GDR fields are reported but have nothing to act on here.
#pragma once

#include <cstdlib>
#include <memory>
#include <string>

namespace mscclpp_amd {

class Env;
std::shared_ptr<Env> env();

class Env {
 public:
  const std::string debug;
  const std::string debugSubsys;
  const std::string debugFile;
  const std::string logLevel;
  const std::string logSubsys;
  const std::string logFile;
  const std::string hcaDevices;
  const std::string ibvSo;
  const std::string ibvMode;
  const std::string hostid;
  const std::string socketFamily;
  const std::string socketIfname;
  const std::string commId;
  const std::string cacheDir;
  const std::string npkitDumpDir;
  const bool cudaIpcUseDefaultStream;
  const std::string ncclSharedLibPath;
  const std::string forceNcclFallbackOperation;
  const bool ncclSymmetricMemory;
  const bool forceDisableNvls;
  const bool forceDisableGdr;
  const int ibGidIndex;

 private:
  static std::string str(const char* name, const std::string& dflt) {
    const char* v = std::getenv(name);
    return v ? std::string(v) : dflt;
  }
  static bool flag(const char* name, bool dflt) {
    const char* v = std::getenv(name);
    return v ? std::string(v) != "0" : dflt;
  }
  static int num(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
  }
  Env()
      : debug(str("MSCCLPP_DEBUG", "")),
        debugSubsys(str("MSCCLPP_DEBUG_SUBSYS", "")),
        debugFile(str("MSCCLPP_DEBUG_FILE", "")),
        logLevel(str("MSCCLPP_LOG_LEVEL", "ERROR")),
        logSubsys(str("MSCCLPP_LOG_SUBSYS", "ALL")),
        logFile(str("MSCCLPP_LOG_FILE", "")),
        hcaDevices(str("MSCCLPP_HCA_DEVICES", "")),
        ibvSo(str("MSCCLPP_IBV_SO", "")),
        ibvMode(str("MSCCLPP_IBV_MODE", "host")),
        hostid(str("MSCCLPP_HOSTID", "")),
        socketFamily(str("MSCCLPP_SOCKET_FAMILY", "")),
        socketIfname(str("MSCCLPP_SOCKET_IFNAME", "")),
        commId(str("MSCCLPP_COMM_ID", "")),
        cacheDir(str("MSCCLPP_CACHE_DIR", str("HOME", "~") + "/.cache/mscclpp")),
        npkitDumpDir(str("MSCCLPP_NPKIT_DUMP_DIR", "")),
        cudaIpcUseDefaultStream(flag("MSCCLPP_CUDAIPC_USE_DEFAULT_STREAM", false)),
        ncclSharedLibPath(str("MSCCLPP_NCCL_LIB_PATH", "")),
        forceNcclFallbackOperation(str("MSCCLPP_FORCE_NCCL_FALLBACK_OPERATION", "")),
        ncclSymmetricMemory(flag("MSCCLPP_NCCL_SYMMETRIC_MEMORY", false)),
        forceDisableNvls(flag("MSCCLPP_FORCE_DISABLE_NVLS", false)),
        forceDisableGdr(flag("MSCCLPP_FORCE_DISABLE_GDR", false)),
        ibGidIndex(num("MSCCLPP_IB_GID_INDEX", 0)) {}
  friend std::shared_ptr<Env> env();
};

inline std::shared_ptr<Env> env() {
  static std::shared_ptr<Env> e(new Env());
  return e;
}

}  // namespace mscclpp_amd
