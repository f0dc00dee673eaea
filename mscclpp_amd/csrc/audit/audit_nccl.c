/* LD_AUDIT redirect: an application (or a framework such as PyTorch) that dlopen()s or links
 * librccl.so / libnccl.so gets libmscclpp_amd.so instead, without relinking and without
 * LD_PRELOAD.  Usage:
 *     LD_AUDIT=/path/to/mscclpp_amd/lib/libmscclpp_amd_audit.so ./app
 *
 * Replaces the reference's src/ext/nccl/audit-shim/audit_nccl.cc:9-17 (la_version / la_objsearch
 * redirecting libnccl.so(.2) and librccl.so(.1) to libmscclpp_nccl.so).  Differences by design:
 *  * the redirect target is an absolute path -- the libmscclpp_amd.so next to this audit library,
 *    or $MSCCLPP_AMD_NCCL_LIB -- so it does not depend on LD_LIBRARY_PATH;
 *  * only the original DT_NEEDED / dlopen name is matched (LA_SER_ORIG), so names the loader
 *    derives while searching are left alone.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <limits.h>
#include <link.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static char g_target[PATH_MAX];

static void resolve_target(void) {
  const char* env = getenv("MSCCLPP_AMD_NCCL_LIB");
  if (env && env[0] && strlen(env) < sizeof(g_target)) {
    strcpy(g_target, env);
    return;
  }
  Dl_info info;
  if (dladdr((void*)&resolve_target, &info) && info.dli_fname) {
    const char* slash = strrchr(info.dli_fname, '/');
    size_t dir = slash ? (size_t)(slash - info.dli_fname) + 1 : 0;
    static const char kLib[] = "libmscclpp_amd.so";
    if (dir + sizeof(kLib) <= sizeof(g_target)) {
      memcpy(g_target, info.dli_fname, dir);
      memcpy(g_target + dir, kLib, sizeof(kLib));
      return;
    }
  }
  strcpy(g_target, "libmscclpp_amd.so");
}

static int is_nccl_name(const char* name) {
  static const char* const kNames[] = {"libnccl.so", "libnccl.so.2", "librccl.so", "librccl.so.1"};
  for (size_t i = 0; i < sizeof(kNames) / sizeof(kNames[0]); ++i)
    if (strcmp(name, kNames[i]) == 0) return 1;
  return 0;
}

__attribute__((visibility("default"))) unsigned int la_version(unsigned int version) {
  (void)version;
  return LAV_CURRENT;
}

__attribute__((visibility("default"))) char* la_objsearch(const char* name, uintptr_t* cookie, unsigned int flag) {
  (void)cookie;
  if (flag == LA_SER_ORIG && name && is_nccl_name(name)) {
    if (!g_target[0]) resolve_target();  /* lazily: the auditor's own namespace is set up by now */
    return g_target;
  }
  return (char*)name;
}
