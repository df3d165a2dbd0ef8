// encoderd.cpp — atgpu-encoderd, the encoder service of one GPU (service.h).
//
// Owns one streaming engine and serves the encode_flac segments of every
// process on the node that asks (over an abstract Unix socket).  Each turn
// of the loop takes every complete request, groups those that share
// options and PCM format, and encodes each group in ONE GPU pass
// (atg_flac_encode_frames_batch): eight track2track conversion processes
// each sending a 64-frame track become one 512-frame batch.  A group that
// fails is retried request by request so an error reaches only its sender.
// Exits after --idle-ms without a connected client (default 3000), after
// taking any connection still queued in the listen backlog.
//
// The socket name is abstract (no file permissions): a connecting process
// of another user is dropped on accept (SO_PEERCRED), and the clients check
// the daemon the same way (service.hip).  Replies are queued per client and
// written from the poll loop without blocking, so a client that stops
// reading holds only its own reply, never the other clients' batches.
//
//   atgpu-encoderd [--device N] [--idle-ms MS]
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "service.h"

namespace {

double now_ms()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

struct Client {
    int fd = -1;
    std::vector<uint8_t> buf; // bytes of the request being received
    size_t need = sizeof(atg_svc_request);
    bool have_header = false;
    bool ready = false;       // a complete request waits in buf
    bool dead = false;
    std::vector<uint8_t> outq; // reply bytes not yet written
    size_t out_off = 0;
};

bool peer_is_me(int fd)
{
    ucred cr;
    socklen_t n = sizeof(cr);
    if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &n) != 0 || n != sizeof(cr))
        return false;
    return cr.uid == getuid();
}

const atg_svc_request &hdr(const Client &c) { return *(const atg_svc_request *)c.buf.data(); }

bool valid_header(const atg_svc_request &q)
{
    if (q.magic != ATG_SVC_MAGIC || q.version != ATG_SVC_VERSION)
        return false;
    if (q.channels < 1 || q.channels > 8 || q.n_frame_sizes > ATG_SVC_MAX_FRAMES)
        return false;
    const uint64_t elem = q.format == ATG_PCM_S16 ? 2 : 4;
    if (q.format != ATG_PCM_S16 && q.format != ATG_PCM_S32)
        return false;
    if (q.pcm_frames > ATG_SVC_MAX_PCM_BYTES || q.pcm_bytes > ATG_SVC_MAX_PCM_BYTES)
        return false;
    return q.pcm_bytes == q.pcm_frames * q.channels * elem;
}

// write what the socket takes now; the rest waits for POLLOUT
void flush(Client &c)
{
    while (!c.dead && c.out_off < c.outq.size()) {
        const ssize_t k = send(c.fd, c.outq.data() + c.out_off, c.outq.size() - c.out_off,
                               MSG_NOSIGNAL | MSG_DONTWAIT);
        if (k < 0) {
            if (errno == EINTR)
                continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK)
                c.dead = true;
            return;
        }
        c.out_off += (size_t)k;
    }
    if (c.out_off == c.outq.size()) {
        c.outq.clear();
        c.outq.shrink_to_fit();
        c.out_off = 0;
    }
}

void put(std::vector<uint8_t> &q, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    q.insert(q.end(), b, b + n);
}

void respond(Client &c, int32_t status, const std::string &msg, const uint8_t *out,
             uint64_t out_bytes, const uint32_t *fb, uint64_t nf)
{
    atg_svc_response r;
    r.status = status;
    const std::string m = msg.substr(0, ATG_SVC_MAX_MSG);
    r.msg_len = (uint32_t)m.size();
    r.out_bytes = status == ATG_OK ? out_bytes : 0;
    r.n_frames = status == ATG_OK ? nf : 0;
    put(c.outq, &r, sizeof(r));
    put(c.outq, m.data(), m.size());
    if (status == ATG_OK) {
        put(c.outq, fb, 4 * nf);
        put(c.outq, out, out_bytes);
    }
    flush(c);
    // ready for the next request
    c.buf.clear();
    c.need = sizeof(atg_svc_request);
    c.have_header = false;
    c.ready = false;
}

// the frames a request's segment holds
uint64_t n_frames_of(const atg_svc_request &q)
{
    if (q.n_frame_sizes)
        return q.n_frame_sizes;
    return q.opts.block_size ? (q.pcm_frames + q.opts.block_size - 1) / q.opts.block_size : 0;
}

// encode a group of requests sharing options and format in one pass
atg_status encode_group(atg_engine *eng, std::vector<Client *> &mem, std::string &err)
{
    const atg_svc_request &q0 = hdr(*mem[0]);
    const uint64_t elem = q0.format == ATG_PCM_S16 ? 2 : 4;
    const uint32_t n = (uint32_t)mem.size();
    std::vector<atg_segment> segs(n);
    uint64_t pcm_frames = 0, cap = 0, nf_total = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const atg_svc_request &q = hdr(*mem[k]);
        atg_segment &g = segs[k];
        g.pcm_offset = pcm_frames;
        g.pcm_frames = q.pcm_frames;
        g.frame_sizes = q.n_frame_sizes ? (const uint32_t *)(mem[k]->buf.data() + sizeof(q)) : nullptr;
        g.n_frame_sizes = q.n_frame_sizes;
        g.first_frame_number = q.first_frame_number;
        pcm_frames += q.pcm_frames;
        const uint64_t b = atg_flac_max_frames_bytes(&q.opts, q.pcm_frames, g.frame_sizes,
                                                     g.n_frame_sizes, q.channels,
                                                     q.bits_per_sample);
        if (!b && q.pcm_frames) {
            err = atg_last_error();
            return ATG_ERR_INVALID;
        }
        cap += (b + 15u) & ~15ull;
        nf_total += n_frames_of(q);
    }
    // one PCM buffer for the batch (the requests' PCM back to back)
    std::vector<uint8_t> pcm(pcm_frames * q0.channels * elem + 16);
    uint64_t at = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const atg_svc_request &q = hdr(*mem[k]);
        std::memcpy(pcm.data() + at, mem[k]->buf.data() + sizeof(q) + 4 * q.n_frame_sizes,
                    q.pcm_bytes);
        at += q.pcm_bytes;
    }
    std::vector<uint8_t> out(cap + 16);
    std::vector<uint64_t> off(n), bytes(n);
    std::vector<uint32_t> fb(nf_total + 1);
    const atg_status st = atg_flac_encode_frames_batch(
        eng, &q0.opts, pcm.data(), (atg_pcm_format)q0.format, segs.data(), n, q0.channels,
        q0.bits_per_sample, q0.sample_rate, out.data(), out.size(), off.data(), bytes.data(),
        fb.data());
    if (st != ATG_OK) {
        err = atg_last_error();
        return st;
    }
    uint64_t f0 = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const uint64_t nf = n_frames_of(hdr(*mem[k]));
        respond(*mem[k], ATG_OK, std::string(), out.data() + off[k], bytes[k], fb.data() + f0, nf);
        f0 += nf;
    }
    return ATG_OK;
}

// accept every queued connection of this user; true if any was taken
bool accept_all(int lfd, std::vector<std::unique_ptr<Client>> &clients)
{
    bool any = false;
    for (;;) {
        const int cfd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (cfd < 0)
            break;
        if (!peer_is_me(cfd)) {
            close(cfd);
            continue;
        }
        auto c = std::make_unique<Client>();
        c->fd = cfd;
        clients.push_back(std::move(c));
        any = true;
    }
    return any;
}

} // namespace

int main(int argc, char **argv)
{
    int device = 0;
    double idle_ms = 3000;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!std::strcmp(argv[i], "--device"))
            device = atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--idle-ms"))
            idle_ms = atof(argv[i + 1]);
    }
    signal(SIGPIPE, SIG_IGN);
    // bind first: a second daemon started by a racing encoder process finds
    // the name taken and leaves
    const int lfd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    if (lfd < 0)
        return 1;
    sockaddr_un a;
    std::memset(&a, 0, sizeof(a));
    a.sun_family = AF_UNIX;
    char name[96];
    const char *env = getenv("ATG_ENCODER_SOCKET");
    if (env && *env)
        snprintf(name, sizeof(name), "%s", env);
    else
        snprintf(name, sizeof(name), ATG_SVC_NAME_FMT, (unsigned)getuid(), device);
    const size_t nl = std::strlen(name);
    std::memcpy(a.sun_path + 1, name, nl);
    if (bind(lfd, (const sockaddr *)&a, (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + nl)) != 0)
        return errno == EADDRINUSE ? 0 : 1;
    if (listen(lfd, 256) != 0)
        return 1;
    atg_engine *eng = nullptr;
    if (atg_engine_create_ex(device, ATG_ENGINE_STREAMING, &eng) != ATG_OK) {
        fprintf(stderr, "atgpu-encoderd: %s\n", atg_last_error());
        return 1;
    }
    std::vector<std::unique_ptr<Client>> clients;
    double last_active = now_ms();
    for (;;) {
        std::vector<pollfd> pf;
        pf.push_back(pollfd{lfd, POLLIN, 0});
        for (auto &c : clients)
            pf.push_back(pollfd{c->fd, (short)(POLLIN | (c->outq.empty() ? 0 : POLLOUT)), 0});
        const int pr = poll(pf.data(), pf.size(), 100);
        if (pr < 0 && errno != EINTR)
            break;
        if (pf[0].revents & POLLIN)
            accept_all(lfd, clients);
        for (size_t i = 1; i < pf.size(); ++i) {
            Client &c = *clients[i - 1];
            if (pf[i].revents & POLLOUT)
                flush(c);
            if (!(pf[i].revents & (POLLIN | POLLHUP | POLLERR)))
                continue;
            // read until the request is complete or the socket is drained
            while (!c.ready && !c.dead) {
                const size_t have = c.buf.size();
                const size_t want = c.need - have;
                c.buf.resize(c.need);
                const ssize_t k = recv(c.fd, c.buf.data() + have, want, 0);
                if (k <= 0) {
                    c.buf.resize(have);
                    if (k == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR))
                        c.dead = true;
                    break;
                }
                c.buf.resize(have + (size_t)k);
                if (c.buf.size() < c.need)
                    continue;
                if (!c.have_header) {
                    if (!valid_header(hdr(c))) {
                        c.dead = true;
                        break;
                    }
                    c.have_header = true;
                    c.need = sizeof(atg_svc_request) + 4 * hdr(c).n_frame_sizes + hdr(c).pcm_bytes;
                    if (c.buf.size() >= c.need)
                        c.ready = true;
                } else {
                    c.ready = true;
                }
            }
        }
        // the turn's batch: every complete request, grouped by format
        std::map<std::string, std::vector<Client *>> groups;
        for (auto &c : clients)
            if (c->ready && !c->dead) {
                const atg_svc_request &q = hdr(*c);
                std::string key((const char *)&q.opts, sizeof(q.opts));
                key.append((const char *)&q.format, 4 * 4); // format, channels, bps, rate
                groups[key].push_back(c.get());
            }
        for (auto &kv : groups) {
            std::string err;
            if (encode_group(eng, kv.second, err) == ATG_OK)
                continue;
            // attribute the failure: each request alone
            for (Client *c : kv.second) {
                std::vector<Client *> one{c};
                std::string e1;
                const atg_status st = encode_group(eng, one, e1);
                if (st != ATG_OK)
                    respond(*c, st, e1, nullptr, 0, nullptr, 0);
            }
        }
        // drop clients that left
        for (size_t i = 0; i < clients.size();) {
            if (clients[i]->dead) {
                close(clients[i]->fd);
                clients.erase(clients.begin() + (std::ptrdiff_t)i);
            } else {
                ++i;
            }
        }
        if (!clients.empty()) {
            last_active = now_ms();
        } else if (now_ms() - last_active > idle_ms) {
            // a connect that landed after the last poll() sits in the
            // backlog: serve it rather than reset it
            pollfd p0{lfd, POLLIN, 0};
            if (poll(&p0, 1, 0) > 0 && accept_all(lfd, clients))
                continue;
            break;
        }
    }
    close(lfd);
    atg_engine_destroy(eng);
    return 0;
}
