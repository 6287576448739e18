// Tiny SIGSEGV reporter for host-side crashes inside native libraries called from Python:
// loaded with ctypes.CDLL after faulthandler.enable(), it prints the native backtrace
// (exported symbols) and then chains to the previous handler (Python's faulthandler stack).
//   gcc -shared -fPIC -O1 bench/segv_bt.c -o bench/segv_bt.so
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction prev;

static void on_segv(int sig, siginfo_t* si, void* uc) {
  void* f[96];
  const int n = backtrace(f, 96);
  const char msg[] = "\n*** SIGSEGV: native backtrace\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(f, n, 2);
  sigaction(SIGSEGV, &prev, NULL);
  if (prev.sa_flags & SA_SIGINFO) prev.sa_sigaction(sig, si, uc);
  else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN) prev.sa_handler(sig);
  else raise(sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &prev);
}
