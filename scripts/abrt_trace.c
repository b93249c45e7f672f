/* Diagnostic only (scripts/rt_exit_probe.py): on SIGABRT / SIGSEGV, print every word of the stack
 * above the handler's frame that points into an executable mapping, as "object+offset" (a stack
 * scan: backtrace() would deadlock when the abort comes from inside _dl_fini, which holds the loader
 * lock). Only raw syscalls and our own formatting run in the handler. Loaded with ctypes by the
 * probe's child, never by the product. Build: gcc -O1 -g -shared -fPIC abrt_trace.c -o abrt_trace.so
 * Offline: the offsets symbolise with llvm-addr2line / nm on the same objects. */
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#define MAXMAP 512
static uintptr_t m_lo[MAXMAP], m_hi[MAXMAP], m_off[MAXMAP];
static char m_name[MAXMAP][160];
static int m_n;
static uintptr_t stk_lo, stk_hi;

static void put(const char* s) { ssize_t r = write(2, s, strlen(s)); (void)r; }
static void puthex(uintptr_t x) {
    char b[19];
    b[0] = '0';
    b[1] = 'x';
    for (int i = 0; i < 16; i++) b[2 + i] = "0123456789abcdef"[(x >> (60 - 4 * i)) & 15];
    b[18] = 0;
    put(b);
}
static uintptr_t hexval(const char** p) {
    uintptr_t v = 0;
    for (;; (*p)++) {
        char c = **p;
        int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
        if (d < 0) return v;
        v = v * 16 + (uintptr_t)d;
    }
}
static void load_maps(void) {
    m_n = 0;
    int fd = open("/proc/self/maps", O_RDONLY);
    if (fd < 0) return;
    static char buf[1 << 20];
    ssize_t k, tot = 0;
    while ((k = read(fd, buf + tot, sizeof buf - 1 - tot)) > 0) tot += k;
    close(fd);
    buf[tot] = 0;
    for (char* ln = buf; *ln;) {
        char* e = strchr(ln, '\n');
        if (e) *e = 0;
        const char* p = ln;
        uintptr_t lo = hexval(&p);
        p++;
        uintptr_t hi = hexval(&p);
        p++;
        int x = p[2] == 'x';
        const char* q = p + 5;
        uintptr_t off = hexval(&q);
        const char* name = strchr(ln, '/');
        if (strstr(ln, "[stack]")) {
            stk_lo = lo;
            stk_hi = hi;
        }
        if (x && name && m_n < MAXMAP) {
            m_lo[m_n] = lo;
            m_hi[m_n] = hi;
            m_off[m_n] = off;
            strncpy(m_name[m_n], name, sizeof m_name[0] - 1);
            m_n++;
        }
        if (!e) break;
        ln = e + 1;
    }
}

static void on_fatal(int sig) {
    put(sig == SIGABRT ? "\n=== SIGABRT stack scan ===\n" : "\n=== SIGSEGV stack scan ===\n");
    load_maps();
    uintptr_t sp = (uintptr_t)__builtin_frame_address(0);
    uintptr_t top = (sp >= stk_lo && sp < stk_hi) ? stk_hi : sp + 16384;
    if (top > sp + 65536) top = sp + 65536;
    int hits = 0;
    for (uintptr_t a = sp & ~(uintptr_t)7; a + 8 <= top && hits < 160; a += 8) {
        uintptr_t w = *(const uintptr_t*)a;
        for (int i = 0; i < m_n; i++) {
            if (w >= m_lo[i] && w < m_hi[i]) {
                put("  ");
                puthex(a - sp);
                put(" ");
                put(m_name[i]);
                put("+");
                puthex(w - m_lo[i] + m_off[i]);
                put("\n");
                hits++;
                break;
            }
        }
    }
    put("=== end ===\n");
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void) {
    signal(SIGABRT, on_fatal);
    signal(SIGSEGV, on_fatal);
}
