// Does an IPC handle of an uncached / plain allocation open in another process (same device)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <unistd.h>
#include <sys/wait.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
    int fd[2], back[2];
    if (pipe(fd) || pipe(back)) return 2;
    pid_t pid = fork();
    if (pid == 0) {
        hipIpcMemHandle_t h[2];
        if (read(fd[0], h, sizeof(h)) != sizeof(h)) return 3;
        CK(hipSetDevice(0));
        void *p[2];
        for (int k = 0; k < 2; ++k) CK(hipIpcOpenMemHandle(&p[k], h[k], hipIpcMemLazyEnablePeerAccess));
        unsigned long long v[2] = {0x1234, 0x5678};
        for (int k = 0; k < 2; ++k) CK(hipMemcpy(p[k], &v[k], 8, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        for (int k = 0; k < 2; ++k) CK(hipIpcCloseMemHandle(p[k]));
        char c = 1;
        if (write(back[1], &c, 1) != 1) return 4;
        return 0;
    }
    CK(hipSetDevice(0));
    void *a = nullptr, *b = nullptr;
    CK(hipExtMallocWithFlags(&a, 4096, hipDeviceMallocUncached));
    CK(hipMalloc(&b, 4096));
    hipIpcMemHandle_t h[2];
    CK(hipIpcGetMemHandle(&h[0], a));
    CK(hipIpcGetMemHandle(&h[1], b));
    if (write(fd[1], h, sizeof(h)) != sizeof(h)) return 5;
    char c;
    if (read(back[0], &c, 1) != 1) return 6;
    int st = 0;
    waitpid(pid, &st, 0);
    unsigned long long v[2] = {0, 0};
    CK(hipMemcpy(&v[0], a, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&v[1], b, 8, hipMemcpyDeviceToHost));
    printf("child exit %d, uncached 0x%llx plain 0x%llx -> %s\n", WEXITSTATUS(st), v[0], v[1],
           (v[0] == 0x1234 && v[1] == 0x5678) ? "IPC OK" : "IPC FAILED");
    return 0;
}
