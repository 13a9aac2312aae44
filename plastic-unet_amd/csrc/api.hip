// Library-level entry points: ABI version, thread-local error text, device info.
#include "common.h"

namespace pu {
thread_local char g_last_error[512] = "";
}

extern "C" int pu_abi_version(void) { return PU_ABI_VERSION; }

extern "C" const char* pu_last_error(void) { return pu::g_last_error; }

extern "C" int pu_device_info(int device, int* num_cu, int* clock_khz, long long* hbm_bytes) {
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return pu::fail(PU_ERR_LAUNCH, "hipGetDeviceProperties: %s", hipGetErrorString(e));
    if (num_cu) *num_cu = prop.multiProcessorCount;
    if (clock_khz) *clock_khz = prop.clockRate;
    if (hbm_bytes) *hbm_bytes = (long long)prop.totalGlobalMem;
    return PU_OK;
}
