// HBM object-store arena: host-side HIP runtime glue for ray_amd's GPU object store.
//
// One process per GPU (the raylet-designated "arena owner") hipMallocs a large
// arena and exports it ONCE with hipIpcGetMemHandle (dmabuf IPC on this ROCm
// stack: HSA_ENABLE_IPC_MODE_LEGACY=0). Every other process on the node opens
// the handle once; from then on a GPU object is just (arena, offset, nbytes) in
// the node's shared-memory object table, and `ray.get` of a GPU tensor is a
// pointer add + DLPack wrap: zero copies, no host bounce. Sub-allocation is
// done by the same native allocator as the host shm store (ray_amd/_native).
#include <hip/hip_runtime.h>
#include <string.h>

#define RA_EXPORT extern "C" __attribute__((visibility("default")))

RA_EXPORT int ra_arena_alloc(int device, size_t bytes, void** ptr, void* handle_out) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return e;
  e = hipMalloc(ptr, bytes);
  if (e != hipSuccess) return e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, *ptr);
  if (e != hipSuccess) return e;
  memcpy(handle_out, &h, sizeof(h));
  return hipSuccess;
}

RA_EXPORT int ra_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

RA_EXPORT int ra_arena_open(int device, const void* handle, void** ptr) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return e;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

RA_EXPORT int ra_arena_close(void* ptr) { return hipIpcCloseMemHandle(ptr); }

RA_EXPORT int ra_arena_free(void* ptr) { return hipFree(ptr); }

RA_EXPORT int ra_copy_async(void* dst, const void* src, size_t n, hipStream_t st) {
  return hipMemcpyAsync(dst, src, n, hipMemcpyDefault, st);
}

RA_EXPORT int ra_stream_sync(hipStream_t st) { return hipStreamSynchronize(st); }

RA_EXPORT int ra_device_count(int* n) { return hipGetDeviceCount(n); }

// Pin an existing host range (e.g. a region of the /dev/shm object store) so
// H2D copies from it run as async DMA at full PCIe rate.
RA_EXPORT int ra_host_register(void* p, size_t n) {
  return hipHostRegister(p, n, hipHostRegisterDefault);
}
RA_EXPORT int ra_host_unregister(void* p) { return hipHostUnregister(p); }
