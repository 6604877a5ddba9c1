/* Diagnosis aid (round 6): on SIGSEGV print the faulting thread's native backtrace
 * (glibc backtrace_symbols_fd) to stderr, then die with the default action.  Loaded by
 * tools/gpu/diag_priority3.py through ctypes before anything touches the GPU. */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>
#include <sys/syscall.h>

static void on_segv(int sig, siginfo_t* si, void* ctx) {
    (void)ctx;
    char msg[160];
    const long tid = syscall(SYS_gettid);
    int n = 0;
    const char* hdr = "\n=== SIGSEGV native backtrace, tid ";
    write(2, hdr, strlen(hdr));
    char num[32];
    int k = 0;
    long t = tid;
    char rev[32];
    do { rev[k++] = (char)('0' + t % 10); t /= 10; } while (t && k < 30);
    while (k) num[n++] = rev[--k];
    num[n++] = '\n';
    write(2, num, n);
    (void)si;
    (void)msg;
    void* fr[64];
    const int m = backtrace(fr, 64);
    backtrace_symbols_fd(fr, m, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigaction(SIGSEGV, &sa, 0);
}
