// Device choice for processes that do not name a device (host code only,
// no HIP call: a track2track conversion process that hands its segments to
// the encoder service never brings up HIP itself).
//
// The reference parallelises track2track by forking one process per track
// (audiotools/__init__.py:5263-5529, track2track:650-669); on an 8-GPU node
// those processes are spread over the GPUs here: ATG_DEVICE, else
// LOCAL_RANK (one process per GPU under torch.distributed), else the next
// device of a node-wide round robin -- a counter in /dev/shm (one per user,
// flock'ed), so `-j 8` conversions land on 8 different GPUs and their
// segments go to 8 per-GPU encoder services (atgpu-encoderd.<uid>.<dev>).
#include "../../include/atgpu.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/file.h>
#include <pthread.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace {

// entries of a comma-separated device list ("0,3,5" -> 3); -1 when unset
int list_count(const char *v)
{
    if (!v)
        return -1;
    int n = 0;
    bool tok = false;
    for (const char *c = v; *c; ++c) {
        if (*c == ',') {
            n += tok;
            tok = false;
        } else if (*c != ' ') {
            tok = true;
        }
    }
    return n + tok;
}

// GPU agents in the KFD topology (nodes with a non-zero gpu_id)
int kfd_gpus()
{
    const char *root = "/sys/class/kfd/kfd/topology/nodes";
    DIR *d = opendir(root);
    if (!d)
        return 0;
    int n = 0;
    while (dirent *e = readdir(d)) {
        if (e->d_name[0] == '.')
            continue;
        const std::string fn = std::string(root) + "/" + e->d_name + "/gpu_id";
        if (FILE *f = std::fopen(fn.c_str(), "r")) {
            unsigned long id = 0;
            if (std::fscanf(f, "%lu", &id) == 1 && id != 0)
                ++n;
            std::fclose(f);
        }
    }
    closedir(d);
    return n;
}

int env_int(const char *name)
{
    const char *v = std::getenv(name);
    if (!v || !*v)
        return -1;
    char *end = nullptr;
    const long x = std::strtol(v, &end, 10);
    return (end && *end == 0 && x >= 0 && x < (1 << 20)) ? (int)x : -1;
}

// the next value of the node-wide counter (-1 if the file cannot be used)
long rr_next()
{
    std::string fn;
    if (const char *v = std::getenv("ATG_RR_FILE"))
        fn = v;
    else
        fn = "/dev/shm/atgpu-rr." + std::to_string((unsigned long)getuid());
    const int fd = open(fn.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (fd < 0)
        return -1;
    long v = -1;
    if (flock(fd, LOCK_EX) == 0) {
        char buf[32] = {0};
        const ssize_t n = pread(fd, buf, sizeof(buf) - 1, 0);
        v = n > 0 ? std::strtol(buf, nullptr, 10) : 0;
        if (v < 0)
            v = 0;
        const int m = std::snprintf(buf, sizeof(buf), "%ld\n", v + 1);
        if (pwrite(fd, buf, (size_t)m, 0) != m || ftruncate(fd, m) != 0)
            v = -1;
        flock(fd, LOCK_UN);
    }
    close(fd);
    return v;
}

std::mutex g_pick_mu;
int g_picked = -1;

// a forked child (track2track's process per track) picks again
struct ForkReset {
    ForkReset() { pthread_atfork(nullptr, nullptr, [] { g_picked = -1; }); }
} g_fork_reset;

} // namespace

extern "C" {

int atg_visible_devices(void)
{
    if (const int n = env_int("ATG_DEVICE_COUNT"); n > 0) // test hook
        return n;
    int n = list_count(std::getenv("HIP_VISIBLE_DEVICES"));
    if (n < 0)
        n = list_count(std::getenv("CUDA_VISIBLE_DEVICES"));
    if (n < 0)
        n = list_count(std::getenv("ROCR_VISIBLE_DEVICES"));
    if (n < 0)
        n = kfd_gpus();
    return n > 0 ? n : 1;
}

int atg_pick_device(void)
{
    std::lock_guard<std::mutex> lk(g_pick_mu);
    if (g_picked >= 0)
        return g_picked;
    int d = env_int("ATG_DEVICE");
    if (d < 0)
        d = env_int("LOCAL_RANK");
    if (d < 0) {
        const int n = atg_visible_devices();
        if (n <= 1) {
            d = 0;
        } else {
            const long v = rr_next();
            d = (int)((v >= 0 ? v : (long)getpid()) % n);
        }
    }
    g_picked = d;
    return d;
}

} // extern "C"
