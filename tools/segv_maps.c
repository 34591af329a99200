/* Diagnostic only (not shipped, not a test): on SIGSEGV, write the faulting
 * address, the interrupted registers, a backtrace and /proc/self/maps to a
 * file, then give the signal back to the handler that was installed before
 * (rocprofv3's), so a host fault inside a library can be attributed to a
 * mapping and a call.  bench.py loads it when PT_SEGV_LOG names the file. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static struct sigaction prev_action;
static char log_path[512];

static void put(int fd, const char* s, int n) {
    while (n > 0) {
        ssize_t w = write(fd, s, (size_t)n);
        if (w <= 0) return;
        s += w;
        n -= (int)w;
    }
}

static void on_segv(int sig, siginfo_t* si, void* ctx) {
    int fd = open(log_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd >= 0) {
        char b[512];
        const ucontext_t* uc = (const ucontext_t*)ctx;
        const greg_t* g = uc->uc_mcontext.gregs;
        int n = snprintf(b, sizeof b,
                         "signal %d addr %p\nrip %llx rsp %llx\nrdi %llx rsi %llx rdx %llx rcx %llx\n"
                         "rax %llx rbx %llx r8 %llx r9 %llx\n",
                         sig, si->si_addr, (unsigned long long)g[REG_RIP], (unsigned long long)g[REG_RSP],
                         (unsigned long long)g[REG_RDI], (unsigned long long)g[REG_RSI],
                         (unsigned long long)g[REG_RDX], (unsigned long long)g[REG_RCX],
                         (unsigned long long)g[REG_RAX], (unsigned long long)g[REG_RBX],
                         (unsigned long long)g[REG_R8], (unsigned long long)g[REG_R9]);
        put(fd, b, n);
        void* bt[64];
        int k = backtrace(bt, 64);
        backtrace_symbols_fd(bt, k, fd);
        put(fd, "--- maps\n", 9);
        int m = open("/proc/self/maps", O_RDONLY);
        if (m >= 0) {
            ssize_t r;
            while ((r = read(m, b, sizeof b)) > 0) put(fd, b, (int)r);
            close(m);
        }
        close(fd);
    }
    /* return into the faulting instruction with the previous handler back in place */
    sigaction(SIGSEGV, &prev_action, NULL);
}

int pt_segv_install(const char* path) {
    strncpy(log_path, path, sizeof log_path - 1);
    void* warm[1];
    backtrace(warm, 1); /* loads libgcc's unwinder now, not inside the handler */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, &prev_action);
}
