// Probe: do CU-masked HIP streams run kernels on this device, and on which XCCs / CUs?
// Each block records (XCC id, HW_ID) once; the host polls for completion with a deadline.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void probe(unsigned *out) {
    if (threadIdx.x == 0) {
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

static bool wait(hipStream_t s, double secs) {
    auto t0 = std::chrono::steady_clock::now();
    while (hipStreamQuery(s) == hipErrorNotReady) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > secs) return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return true;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", cus);
    fflush(stdout);
    unsigned *out;
    hipMalloc(&out, 4096 * 8);
    const int lo_counts[] = {8, 16, 40};
    for (int nc : lo_counts) {
        for (int hi = 0; hi < 2; ++hi) {
            std::vector<uint32_t> m((cus + 31) / 32, 0u);
            for (int i = 0; i < cus; ++i)
                if ((i < nc) != (hi == 1)) m[i / 32] |= 1u << (i % 32);
            hipStream_t s;
            hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data());
            printf("mask %s%d: create %s\n", hi ? "not-low" : "low", nc, hipGetErrorString(e));
            fflush(stdout);
            if (e != hipSuccess) continue;
            std::vector<uint32_t> got(m.size(), 0u);
            hipExtStreamGetCUMask(s, (uint32_t)got.size(), got.data());
            printf("  get mask word0 %08x word1 %08x\n", got[0], got.size() > 1 ? got[1] : 0);
            const int blocks = hi ? 64 : nc;
            hipMemsetAsync(out, 0xff, 4096 * 8, s);
            probe<<<blocks, 512, 0, s>>>(out);
            const bool ok = wait(s, 5.0);
            printf("  kernel %d blocks: %s\n", blocks, ok ? "done" : "NOT DONE after 5 s");
            fflush(stdout);
            if (!ok) return 2;
            std::vector<unsigned> h(2 * blocks);
            hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
            printf("  (xcc,cu,se):");
            for (int b = 0; b < blocks && b < 24; ++b)
                printf(" (%u,%u,%u)", h[2 * b], (h[2 * b + 1] >> 8) & 15, (h[2 * b + 1] >> 13) & 7);
            printf("\n");
            fflush(stdout);
            hipStreamDestroy(s);
        }
    }
    printf("probe done\n");
    return 0;
}
