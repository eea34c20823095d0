// api.cpp -- library-wide C ABI entry points (version, errors, devices).
#include <cstdlib>
#include <string>

#include "fh_common.h"

namespace fh {

namespace {
thread_local std::string g_last_error;
}

void set_last_error(const std::string &m) { g_last_error = m; }

thread_local Probe *t_probe = nullptr;

int pick_device(const fh_config *cfg, uint64_t shard_id) {
  int count = 0;
  FH_HIP(hipGetDeviceCount(&count));
  FH_CHECK(count > 0, FH_EHIP, "no HIP device visible");
  if (cfg && cfg->device >= 0) {
    FH_CHECK(cfg->device < count, FH_EINVAL, "device ordinal out of range");
    return cfg->device;
  }
  if (const char *env = std::getenv("FANTOCH_HIP_DEVICE")) {
    int d = std::atoi(env);
    FH_CHECK(d >= 0 && d < count, FH_EINVAL, "FANTOCH_HIP_DEVICE out of range");
    return d;
  }
  return int(shard_id % uint64_t(count));
}

}  // namespace fh

extern "C" {

const char *fh_version(void) { return "fantoch_hip 0.1.0 (gfx950, abi 1)"; }

const char *fh_last_error(void) { return fh::g_last_error.c_str(); }

fh_status fh_device_count(int *out) {
  FH_API_BEGIN
  FH_CHECK(out, FH_EINVAL, "null argument");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  *out = e == hipSuccess ? c : 0;
  FH_API_END
}

}  // extern "C"
