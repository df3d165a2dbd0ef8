// service.hip — client side of the encoder service (service.h): host code
// only.  atg_service_encode_frames has atg_flac_encode_frames' contract; the
// segment travels over the service's Unix socket and is encoded by the
// process that owns the GPU engine (atgpu-encoderd, encoderd.cpp).
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <cstring>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "service.h"

struct atg_service {
    int fd = -1;
    int device = 0;
};

namespace {

thread_local std::string g_svc_err;

atg_status sfail(atg_status s, const std::string &m)
{
    g_svc_err = m;
    return s;
}

// the abstract socket address of `device`'s service
socklen_t service_addr(int device, sockaddr_un &a)
{
    std::memset(&a, 0, sizeof(a));
    a.sun_family = AF_UNIX;
    char name[96];
    const char *env = getenv("ATG_ENCODER_SOCKET");
    if (env && *env)
        snprintf(name, sizeof(name), "%s", env);
    else
        snprintf(name, sizeof(name), ATG_SVC_NAME_FMT, (unsigned)getuid(), device);
    const size_t n = strlen(name);
    std::memcpy(a.sun_path + 1, name, n); // sun_path[0] = 0: abstract namespace
    return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
}

// abstract sockets carry no file permissions: whoever binds the name first
// owns it.  The peer must be a process of this user (SO_PEERCRED), or the
// socket is dropped -- PCM is never sent to, and frames never taken from,
// another user's process.  (The daemon checks its clients the same way.)
bool peer_is_me(int fd)
{
    ucred cr;
    socklen_t n = sizeof(cr);
    if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &n) != 0 || n != sizeof(cr))
        return false;
    return cr.uid == getuid();
}

// -1: nothing listens; -2: a listener of another user holds the name
int try_connect(int device)
{
    const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0)
        return -1;
    sockaddr_un a;
    const socklen_t len = service_addr(device, a);
    if (connect(fd, (const sockaddr *)&a, len) == 0) {
        if (peer_is_me(fd))
            return fd;
        close(fd);
        return -2;
    }
    close(fd);
    return -1;
}

// has this process opened the GPU itself?  Then it must not exec the
// service (a process that initialised the GPU may not exec another program)
bool gpu_opened()
{
    FILE *f = fopen("/proc/self/maps", "r");
    if (!f)
        return true; // unknown: do not spawn
    char line[512];
    bool found = false;
    while (!found && fgets(line, sizeof(line), f))
        found = strstr(line, "/dev/kfd") != nullptr;
    fclose(f);
    return found;
}

// atgpu-encoderd beside libatgpu.so (or ATG_ENCODERD), started as a
// daemon: double fork + setsid, stdio on /dev/null and no inherited file
// descriptors, so it outlives the encoder process that started it and holds
// none of its pipes
bool spawn_service(int device)
{
    std::string path;
    const char *env = getenv("ATG_ENCODERD");
    if (env && *env) {
        path = env;
    } else {
        Dl_info info;
        if (!dladdr((void *)&spawn_service, &info) || !info.dli_fname)
            return false;
        path = info.dli_fname;
        const size_t slash = path.rfind('/');
        path = (slash == std::string::npos ? std::string(".") : path.substr(0, slash)) +
               "/atgpu-encoderd";
    }
    if (access(path.c_str(), X_OK) != 0)
        return false;
    char dev[16];
    snprintf(dev, sizeof(dev), "%d", device);
    const pid_t p = fork();
    if (p < 0)
        return false;
    if (p == 0) {
        setsid();
        const pid_t q = fork();
        if (q != 0)
            _exit(0);
        const int nul = open("/dev/null", O_RDWR);
        if (nul >= 0) {
            dup2(nul, 0);
            dup2(nul, 1);
            dup2(nul, 2);
        }
        const long maxfd = sysconf(_SC_OPEN_MAX);
        for (long k = 3; k < (maxfd > 0 ? maxfd : 1024); ++k)
            close((int)k);
        execl(path.c_str(), path.c_str(), "--device", dev, (char *)nullptr);
        _exit(127);
    }
    int st = 0;
    while (waitpid(p, &st, 0) < 0 && errno == EINTR) {
    }
    return true;
}

bool send_all(int fd, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    while (n) {
        const ssize_t k = send(fd, b, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR)
                continue;
            return false;
        }
        b += k;
        n -= (size_t)k;
    }
    return true;
}

double mono_ms()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

// receive exactly n bytes before the absolute deadline (CLOCK_MONOTONIC ms);
// false on EOF, error or timeout
bool recv_all(int fd, void *p, size_t n, double deadline)
{
    uint8_t *b = (uint8_t *)p;
    while (n) {
        const double left = deadline - mono_ms();
        if (left <= 0)
            return false;
        pollfd pf{fd, POLLIN, 0};
        const int pr = poll(&pf, 1, left > 1e9 ? 1000000000 : (int)left + 1);
        if (pr < 0 && errno == EINTR)
            continue;
        if (pr <= 0)
            return false;
        const ssize_t k = recv(fd, b, n, 0);
        if (k < 0 && (errno == EINTR || errno == EAGAIN))
            continue;
        if (k <= 0)
            return false;
        b += k;
        n -= (size_t)k;
    }
    return true;
}

void sleep_ms(unsigned ms)
{
    timespec ts{(time_t)(ms / 1000), (long)(ms % 1000) * 1000000L};
    nanosleep(&ts, nullptr);
}

// how long a segment may take the service: a fixed allowance for HIP
// start-up and the batch it joins, plus its PCM at a rate far below any
// real encode (50 MB/s); the service's stall past this is treated as its
// loss, and the caller encodes on an engine of its own
double segment_deadline_ms(uint64_t pcm_bytes)
{
    const char *env = getenv("ATG_SERVICE_TIMEOUT_MS");
    const double base = env && *env ? atof(env) : 30000.0;
    return mono_ms() + base + (double)pcm_bytes / 50e3;
}

// the connection is out of step (timeout, malformed reply): drop it
atg_status lose(atg_service *s, const char *m)
{
    if (s->fd >= 0)
        close(s->fd);
    s->fd = -1;
    return sfail(ATG_ERR_DEVICE, m);
}

} // namespace

extern "C" {

const char *atg_service_last_error(void) { return g_svc_err.c_str(); }

atg_status atg_service_connect(int device, int spawn, atg_service **out)
{
    if (!out)
        return sfail(ATG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int fd = try_connect(device);
    if (fd == -2)
        return sfail(ATG_ERR_DEVICE, "the encoder service's name is held by another user");
    if (fd < 0 && spawn) {
        if (gpu_opened())
            return sfail(ATG_ERR_DEVICE, "this process has opened the GPU: not starting the "
                                         "encoder service from it");
        if (!spawn_service(device))
            return sfail(ATG_ERR_DEVICE, "atgpu-encoderd not found or not started");
        // the service binds its socket first, then brings up HIP; connects
        // queue in its backlog meanwhile
        for (unsigned waited = 0, step = 2; fd == -1 && waited < 30000; waited += step) {
            sleep_ms(step);
            fd = try_connect(device);
            step = step < 64 ? 2 * step : 64;
        }
        if (fd == -2)
            return sfail(ATG_ERR_DEVICE, "the encoder service's name is held by another user");
    }
    if (fd < 0)
        return sfail(ATG_ERR_DEVICE, "no encoder service for this device");
    atg_service *s = new atg_service();
    s->fd = fd;
    s->device = device;
    *out = s;
    return ATG_OK;
}

void atg_service_close(atg_service *s)
{
    if (!s)
        return;
    if (s->fd >= 0)
        close(s->fd);
    delete s;
}

atg_status atg_service_encode_frames(atg_service *s, const atg_flac_options *opts,
                                     const void *pcm, atg_pcm_format format, uint64_t pcm_frames,
                                     const uint32_t *frame_sizes, uint64_t n_frame_sizes,
                                     uint32_t channels, uint32_t bps, uint32_t rate,
                                     uint64_t first_frame_number, uint8_t *out, uint64_t out_cap,
                                     uint64_t *out_bytes, uint32_t *frame_bytes)
{
    if (!s || !opts || (!pcm && pcm_frames) || !out_bytes)
        return sfail(ATG_ERR_INVALID, "NULL argument");
    if (s->fd < 0)
        return sfail(ATG_ERR_DEVICE, "encoder service connection lost");
    if (channels < 1 || channels > 8 || n_frame_sizes > ATG_SVC_MAX_FRAMES ||
        (frame_sizes == nullptr && n_frame_sizes))
        return sfail(ATG_ERR_INVALID, "invalid segment");
    const uint64_t elem = format == ATG_PCM_S16 ? 2 : 4;
    atg_svc_request q;
    std::memset(&q, 0, sizeof(q));
    q.magic = ATG_SVC_MAGIC;
    q.version = ATG_SVC_VERSION;
    q.opts = *opts;
    q.format = (uint32_t)format;
    q.channels = channels;
    q.bits_per_sample = bps;
    q.sample_rate = rate;
    q.pcm_frames = pcm_frames;
    q.n_frame_sizes = frame_sizes ? n_frame_sizes : 0;
    q.first_frame_number = first_frame_number;
    q.pcm_bytes = pcm_frames * channels * elem;
    if (q.pcm_bytes > ATG_SVC_MAX_PCM_BYTES)
        return sfail(ATG_ERR_UNSUPPORTED, "segment too large for the encoder service");
    // the frames the reply must describe: one per given size, else one per
    // block (the service's own count, encoderd.cpp n_frames_of)
    const uint64_t want_frames =
        q.n_frame_sizes ? q.n_frame_sizes
                        : (opts->block_size ? (pcm_frames + opts->block_size - 1) / opts->block_size
                                            : 0);
    const double deadline = segment_deadline_ms(q.pcm_bytes);
    if (!send_all(s->fd, &q, sizeof(q)) ||
        (q.n_frame_sizes && !send_all(s->fd, frame_sizes, 4 * q.n_frame_sizes)) ||
        (q.pcm_bytes && !send_all(s->fd, pcm, q.pcm_bytes)))
        return lose(s, "encoder service connection lost (send)");
    atg_svc_response r;
    if (!recv_all(s->fd, &r, sizeof(r), deadline))
        return lose(s, "encoder service lost or timed out (receive)");
    if (r.msg_len > ATG_SVC_MAX_MSG)
        return lose(s, "encoder service: malformed response");
    std::string msg(r.msg_len, '\0');
    if (r.msg_len && !recv_all(s->fd, &msg[0], r.msg_len, deadline))
        return lose(s, "encoder service lost or timed out (receive)");
    if (r.status != ATG_OK) {
        if (r.n_frames || r.out_bytes)
            return lose(s, "encoder service: malformed response");
        return sfail((atg_status)r.status, msg);
    }
    // the reply is checked against the request before any byte of it is
    // stored: exactly the requested frame count (frame_bytes holds that many),
    // frame sizes that add up to out_bytes, and out_bytes within the bound
    // the segment's options allow
    if (r.n_frames != want_frames)
        return lose(s, "encoder service: response frame count differs from the request");
    const uint64_t bound = atg_flac_max_frames_bytes(opts, pcm_frames, q.n_frame_sizes ? frame_sizes
                                                                                       : nullptr,
                                                     q.n_frame_sizes, channels, bps);
    if (r.out_bytes > bound)
        return lose(s, "encoder service: response larger than the segment's bound");
    std::vector<uint32_t> fb((size_t)r.n_frames);
    if (r.n_frames && !recv_all(s->fd, fb.data(), 4 * fb.size(), deadline))
        return lose(s, "encoder service lost or timed out (receive)");
    uint64_t sum = 0;
    for (uint32_t b : fb)
        sum += b;
    if (sum != r.out_bytes)
        return lose(s, "encoder service: frame sizes do not add up to the response");
    if (r.out_bytes > out_cap) {
        // drain the frames to keep the stream in step, then report
        std::vector<uint8_t> sink((size_t)r.out_bytes);
        if (!recv_all(s->fd, sink.data(), sink.size(), deadline))
            return lose(s, "encoder service lost or timed out (receive)");
        *out_bytes = r.out_bytes;
        return sfail(ATG_ERR_CAPACITY, "output buffer too small for the segment's frames");
    }
    if (r.out_bytes && !recv_all(s->fd, out, r.out_bytes, deadline))
        return lose(s, "encoder service lost or timed out (receive)");
    *out_bytes = r.out_bytes;
    if (frame_bytes && r.n_frames)
        std::memcpy(frame_bytes, fb.data(), 4 * fb.size());
    return ATG_OK;
}

} // extern "C"
