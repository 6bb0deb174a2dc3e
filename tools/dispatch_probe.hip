// dispatch_probe.hip -- how much of the per-call fixed cost is the HIP
// launch path (tuning tool, not part of the library).
//   hipcc --offload-arch=gfx950 -O2 tools/dispatch_probe.hip -lhsa-runtime64 -o tools/dispatch_probe
//   hipcc --offload-arch=gfx950 -O2 --genco tools/dispatch_probe.hip -o tools/dispatch_probe.hsaco
//
// One "call" = dispatch a one-wave kernel that stores a host-coherent flag,
// then spin on the flag (the library's blocking protocol). Per call: the
// host time inside the launch API, and the round trip launch -> flag seen.
//   hip     : hipExtLaunchKernelGGL on a blocking stream (the library's path)
//   hsa     : the same kernel from the .hsaco, an AQL packet written straight
//             into a queue of our own (hsa_queue_create), kernarg in host
//             memory or in fine-grained device memory
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
#define HCHECK(x) do { hsa_status_t s = (x); if (s != HSA_STATUS_SUCCESS) { \
    const char *m = nullptr; hsa_status_string(s, &m); fprintf(stderr, "%s: %s\n", #x, m ? m : "?"); exit(1); } } while (0)

struct Args {
    unsigned *flag;
    unsigned epoch;
};

extern "C" __global__ __launch_bounds__(64) void probe_k(Args a) {
    if (threadIdx.x == 0) __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the same kernel with a larger argument block (the fused kernel's is 1.5 KiB)
template <int PAD>
struct BigArgs {
    unsigned *flag;
    unsigned epoch;
    unsigned long long pad[PAD];
};
template <int PAD>
__global__ __launch_bounds__(64) void probe_big_k(BigArgs<PAD> a) {
    if (threadIdx.x == 0) __hip_atomic_store(a.flag, a.epoch + (unsigned)a.pad[PAD - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// main() is host-only below: instantiate the kernels where the device pass sees them
template __global__ void probe_big_k<4>(BigArgs<4>);
template __global__ void probe_big_k<64>(BigArgs<64>);
template __global__ void probe_big_k<188>(BigArgs<188>);
template __global__ void probe_big_k<380>(BigArgs<380>);

#ifndef __HIP_DEVICE_COMPILE__
static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static void report(const char *name, std::vector<double> &api, std::vector<double> &rt) {
    printf("%-40s api %6.2f us   round trip %6.2f us  (p10 %6.2f)\n", name, med(api) * 1e6, med(rt) * 1e6,
           [&] { auto v = rt; std::sort(v.begin(), v.end()); return v[v.size() / 10]; }() * 1e6);
}

static inline void spin(volatile unsigned *flag, unsigned want) {
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != want) {
    }
}

static hsa_agent_t g_gpu;
static hsa_amd_memory_pool_t g_kernarg_pool, g_fine_dev_pool;
static bool g_have_kernarg = false, g_have_fine = false;

static hsa_status_t pick_pool(hsa_amd_memory_pool_t pool, void *data) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    const bool is_gpu = data != nullptr;
    if (!is_gpu && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_kernarg) {
        g_kernarg_pool = pool;
        g_have_kernarg = true;
    }
    if (is_gpu && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !g_have_fine) {
        g_fine_dev_pool = pool;
        g_have_fine = true;
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t pick_agent(hsa_agent_t agent, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) {
        g_gpu = agent;
        hsa_amd_agent_iterate_memory_pools(agent, pick_pool, (void *)1);
    } else if (t == HSA_DEVICE_TYPE_CPU) {
        hsa_amd_agent_iterate_memory_pools(agent, pick_pool, nullptr);
    }
    return HSA_STATUS_SUCCESS;
}

int main(int argc, char **argv) {
    const char *hsaco = argc > 1 ? argv[1] : "tools/dispatch_probe.hsaco";
    const int calls = 20000;
    CHECK(hipSetDevice(0));
    unsigned *flag;
    CHECK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    unsigned epoch = 0;
    {
        std::vector<double> api, rt;
        for (int i = 0; i < calls + 200; ++i) {
            Args a{flag, ++epoch};
            const double t0 = now();
            hipExtLaunchKernelGGL(probe_k, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0, a);
            const double t1 = now();
            spin(flag, epoch);
            const double t2 = now();
            if (i >= 200) {
                api.push_back(t1 - t0);
                rt.push_back(t2 - t0);
            }
        }
        report("hip: hipExtLaunchKernelGGL", api, rt);
    }
    CHECK(hipStreamSynchronize(st));
    auto big = [&](auto tag, const char *name) {
        constexpr int PAD = decltype(tag)::value;
        std::vector<double> api, rt;
        for (int i = 0; i < calls + 200; ++i) {
            BigArgs<PAD> a{};
            a.flag = flag;
            a.epoch = ++epoch;
            const double t0 = now();
            hipExtLaunchKernelGGL(probe_big_k<PAD>, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0, a);
            const double t1 = now();
            spin(flag, epoch);
            const double t2 = now();
            if (i >= 200) {
                api.push_back(t1 - t0);
                rt.push_back(t2 - t0);
            }
        }
        report(name, api, rt);
    };
    big(std::integral_constant<int, 4>{}, "hip: 48 B of kernel arguments");
    big(std::integral_constant<int, 64>{}, "hip: 528 B of kernel arguments");
    big(std::integral_constant<int, 188>{}, "hip: 1.5 KiB of kernel arguments");
    big(std::integral_constant<int, 380>{}, "hip: 3 KiB of kernel arguments");
    CHECK(hipStreamSynchronize(st));
    if (argc > 2) return 0;  // HIP part only

    // ---- HSA direct dispatch
    HCHECK(hsa_init());
    HCHECK(hsa_iterate_agents(pick_agent, nullptr));
    if (g_gpu.handle == 0 || !g_have_kernarg) {
        fprintf(stderr, "no GPU agent / kernarg pool\n");
        return 1;
    }
    FILE *f = fopen(hsaco, "rb");
    if (!f) {
        perror(hsaco);
        return 1;
    }
    std::vector<char> blob;
    {
        fseek(f, 0, SEEK_END);
        blob.resize(ftell(f));
        fseek(f, 0, SEEK_SET);
        if (fread(blob.data(), 1, blob.size(), f) != blob.size()) return 1;
        fclose(f);
    }
    hsa_code_object_reader_t reader;
    HCHECK(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &reader));
    hsa_executable_t exe;
    HCHECK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    HCHECK(hsa_executable_load_agent_code_object(exe, g_gpu, reader, nullptr, nullptr));
    HCHECK(hsa_executable_freeze(exe, nullptr));
    hsa_executable_symbol_t sym;
    HCHECK(hsa_executable_get_symbol_by_name(exe, "probe_k.kd", &g_gpu, &sym));
    uint64_t kobj;
    uint32_t kasz, gsz, psz;
    HCHECK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
    HCHECK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kasz));
    HCHECK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gsz));
    HCHECK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &psz));
    printf("probe_k: kernarg %u B, group %u, private %u\n", kasz, gsz, psz);
    hsa_queue_t *q;
    HCHECK(hsa_queue_create(g_gpu, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));

    const int ring = 64;
    const size_t kstride = (kasz + 255) / 256 * 256;
    for (int variant = 0; variant < 3; ++variant) {
        char *kargs = nullptr;
        if (variant == 0) {
            HCHECK(hsa_amd_memory_pool_allocate(g_kernarg_pool, kstride * ring, 0, (void **)&kargs));
            HCHECK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, kargs));
        } else if (variant == 1) {
            if (!g_have_fine) continue;
            HCHECK(hsa_amd_memory_pool_allocate(g_fine_dev_pool, kstride * ring, 0, (void **)&kargs));
        } else {
            CHECK(hipHostMalloc((void **)&kargs, kstride * ring, hipHostMallocCoherent | hipHostMallocMapped));
        }
        std::vector<double> api, rt;
        char zero[4096] = {0};
        for (int i = 0; i < calls + 200; ++i) {
            Args a{flag, ++epoch};
            const double t0 = now();
            char *ka = kargs + (size_t)(i % ring) * kstride;
            if (variant == 1) {
                // device memory: host writes go over PCIe (mapped fine-grained)
                memcpy(zero, &a, sizeof a);
                memcpy(ka, zero, kasz);
            } else {
                memset(ka, 0, kasz);
                memcpy(ka, &a, sizeof a);
            }
            const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
            hsa_kernel_dispatch_packet_t *pkt = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx % q->size);
            pkt->workgroup_size_x = 64;
            pkt->workgroup_size_y = 1;
            pkt->workgroup_size_z = 1;
            pkt->grid_size_x = 64;
            pkt->grid_size_y = 1;
            pkt->grid_size_z = 1;
            pkt->private_segment_size = psz;
            pkt->group_segment_size = gsz;
            pkt->kernel_object = kobj;
            pkt->kernarg_address = ka;
            pkt->reserved2 = 0;
            pkt->completion_signal.handle = 0;
            const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                    (1 << HSA_PACKET_HEADER_BARRIER) |
                                    (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                    (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
            const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
            __atomic_store_n((uint32_t *)pkt, header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
            hsa_signal_store_screlease(q->doorbell_signal, idx);
            const double t1 = now();
            spin(flag, epoch);
            const double t2 = now();
            if (i >= 200) {
                api.push_back(t1 - t0);
                rt.push_back(t2 - t0);
            }
        }
        report(variant == 0 ? "hsa: AQL, kernarg pool (host)" : variant == 1 ? "hsa: AQL, fine-grained device kernarg"
                                                                             : "hsa: AQL, hipHostMalloc kernarg",
               api, rt);
    }
    // again HIP, to see that the second queue did not change it
    {
        std::vector<double> api, rt;
        for (int i = 0; i < calls + 200; ++i) {
            Args a{flag, ++epoch};
            const double t0 = now();
            hipExtLaunchKernelGGL(probe_k, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0, a);
            const double t1 = now();
            spin(flag, epoch);
            const double t2 = now();
            if (i >= 200) {
                api.push_back(t1 - t0);
                rt.push_back(t2 - t0);
            }
        }
        report("hip again", api, rt);
    }
    CHECK(hipStreamSynchronize(st));
    hsa_queue_destroy(q);
    return 0;
}
#endif
