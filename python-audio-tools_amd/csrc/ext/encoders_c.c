/*
 * encoders_c.c — audiotools._encoders_c: the reference's CPython encoder
 * entry point, compiled, over libatgpu's C ABI (include/atgpu.h).
 *
 * encode_flac(filename, pcmreader, block_size, max_lpc_order,
 *             min_residual_partition_order, max_residual_partition_order,
 *             mid_side=0, adaptive_mid_side=0, exhaustive_model_search=0,
 *             disable_verbatim_subframes=0, disable_constant_subframes=0,
 *             disable_fixed_subframes=0, disable_lpc_subframes=0,
 *             padding_size=4096) -> [(byte_offset, pcm_frames), ...]
 *
 * Same argument parsing as the reference (src/encoders/flac.c:52-108,
 * "sOIIII|iiiiiiiI"; registered src/encoders.h:65-67), same frame loop:
 * every pcmreader.read(block_size) becomes one FLAC frame
 * (flac.c:244-274), an empty read ends the stream, read() results must be
 * pcm.FrameList (TypeError, pcmconv.c:244-248) and read() exceptions
 * propagate.  The output file is opened first (IOError with errno and
 * filename, flac.c:114-116); the stream header is written before the frames
 * and rewritten with the final STREAMINFO at the end (flac.c:208-238,
 * 276-279); the reader is closed on success (flac.c:282).
 *
 * The frames are encoded on the GPU in bounded segments of SEGMENT_FRAMES
 * frames (atg_flac_encode_frames), with the GIL released around each
 * segment as the reference releases it around each frame (flac.c:255-270);
 * the STREAMINFO MD5 of the PCM bytes (what the reference's read callback
 * hashes, pcmconv.c:266-291; RFC 1321 below) runs over each segment on a
 * host thread while the GPU encodes it.  Host memory stays bounded by one
 * segment.  The engine is a streaming one (ATG_ENGINE_STREAMING): one
 * process per track, as track2track runs encoders, holds two HIP streams.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/atgpu.h"

#define SEGMENT_FRAMES 256 /* the most frames per GPU call */
static unsigned g_segment_frames = SEGMENT_FRAMES; /* _set_segment_frames (tests) */

#include "md5_host.h"

/* the MD5 bytes of a segment: FrameList.to_bytes(little_endian, signed) of
   its samples (flac.c:187-188), from the segment's int16 / int32 container */
typedef struct {
    md5_ctx *md5;
    const uint8_t *pcm;
    size_t samples, elem;
    unsigned width;
} md5_job;

static void *md5_segment(void *arg)
{
    md5_job *j = (md5_job *)arg;
    if (j->width == j->elem) { /* 16-bit in int16, 32-bit in int32: as stored */
        md5_update(j->md5, j->pcm, j->samples * j->elem);
        return NULL;
    }
    uint8_t tmp[4096];
    size_t tl = 0;
    for (size_t i = 0; i < j->samples; ++i) {
        const uint8_t *x = j->pcm + i * j->elem; /* little-endian container */
        for (unsigned k = 0; k < j->width; ++k)
            tmp[tl++] = x[k];
        if (tl + 4 > sizeof(tmp)) {
            md5_update(j->md5, tmp, tl);
            tl = 0;
        }
    }
    md5_update(j->md5, tmp, tl);
    return NULL;
}

/* ------------------------------------------------------------- module */
static PyObject *g_framelist_type; /* audiotools.pcm.FrameList */
static atg_engine *g_eng;      /* this process's own engine (no service) */
static atg_service *g_svc;     /* the encoder service (atgpu-encoderd) */
static int g_svc_mode = -1;    /* -1 undecided, 0 own engine, 1 service */

/* ATG_DEVICE, LOCAL_RANK, else a node-wide round robin over the visible
   GPUs (atg_pick_device): track2track's processes spread over the node */
static int engine_device(void)
{
    return atg_pick_device();
}

static PyObject *raise_atg(atg_status st)
{
    PyErr_SetString(st == ATG_ERR_INVALID || st == ATG_ERR_UNSUPPORTED ? PyExc_ValueError
                                                                        : PyExc_RuntimeError,
                    atg_last_error());
    return NULL;
}

typedef struct {
    FILE *f;
    atg_flac_options o;
    unsigned channels, bps, rate;
    /* the segment being collected: interleaved samples (int16 for <= 16
       bits, int32 otherwise) and the frame count of every read */
    uint8_t *pcm;
    size_t pcm_cap, pcm_len; /* bytes */
    uint32_t sizes[SEGMENT_FRAMES];
    unsigned n_sizes;
    uint64_t frame_no, offset, total;
    uint32_t min_fs, max_fs;
    uint8_t *out;
    size_t out_cap;
    uint32_t *frame_bytes;
    PyObject *list;
    md5_ctx md5;
} enc_state;

/* where this process's segments are encoded: the encoder service (one
   process per GPU owning the engine, started on first use; a track2track
   conversion process then never brings up HIP itself) unless
   ATG_ENCODER_SERVICE=off, or the service cannot be reached -- then an
   engine of this process's own.  Decided once per process. */
static int choose_backend(void)
{
    if (g_svc_mode < 0) {
        const char *v = getenv("ATG_ENCODER_SERVICE");
        g_svc_mode = !(v && (!strcmp(v, "off") || !strcmp(v, "0")));
        if (g_svc_mode && atg_service_connect(engine_device(), 1, &g_svc) != ATG_OK)
            g_svc_mode = 0;
    }
    if (!g_svc_mode && !g_eng) {
        const atg_status st = atg_engine_create_ex(engine_device(), ATG_ENGINE_STREAMING, &g_eng);
        if (st != ATG_OK) {
            raise_atg(st);
            return -1;
        }
    }
    return 0;
}

/* encode and write the collected segment; appends to the offsets list */
static int flush_segment(enc_state *s)
{
    if (!s->n_sizes)
        return 0;
    if (choose_backend() < 0)
        return -1;
    const size_t elem = s->bps <= 16 ? 2 : 4;
    const uint64_t frames = s->pcm_len / (elem * s->channels);
    uint64_t cap = atg_flac_max_frames_bytes(&s->o, frames, s->sizes, s->n_sizes,
                                             s->channels, s->bps);
    if (!cap) {
        PyErr_SetString(PyExc_ValueError, "invalid encoder options");
        return -1;
    }
    cap = (cap + 15u) & ~(uint64_t)15u; /* the engine packs segments 16-byte aligned */
    if (cap > s->out_cap) {
        uint8_t *p = (uint8_t *)PyMem_Realloc(s->out, cap);
        if (!p) {
            PyErr_NoMemory();
            return -1;
        }
        s->out = p;
        s->out_cap = cap;
    }
    uint64_t nb = 0;
    atg_status st;
    md5_job mj = {&s->md5, s->pcm, (size_t)(frames * s->channels), elem, (s->bps + 7) / 8};
    const atg_pcm_format fmt = s->bps <= 16 ? ATG_PCM_S16 : ATG_PCM_S32;
    const char *svc_err = NULL;
    int lost = 0;
    Py_BEGIN_ALLOW_THREADS
    pthread_t hasher;
    const int threaded = pthread_create(&hasher, NULL, md5_segment, &mj) == 0;
    if (!threaded)
        md5_segment(&mj);
    if (g_svc) {
        st = atg_service_encode_frames(g_svc, &s->o, s->pcm, fmt, frames, s->sizes, s->n_sizes,
                                       s->channels, s->bps, s->rate, s->frame_no, s->out,
                                       s->out_cap, &nb, s->frame_bytes);
        if (st != ATG_OK)
            svc_err = atg_service_last_error();
        lost = st == ATG_ERR_DEVICE; /* the service went away: this process's own engine */
    } else {
        st = atg_flac_encode_frames(g_eng, &s->o, s->pcm, fmt, frames, s->sizes, s->n_sizes,
                                    s->channels, s->bps, s->rate, s->frame_no, s->out,
                                    s->out_cap, &nb, s->frame_bytes);
    }
    if (threaded)
        pthread_join(hasher, NULL);
    Py_END_ALLOW_THREADS
    if (lost) {
        atg_service_close(g_svc);
        g_svc = NULL;
        g_svc_mode = 0;
        svc_err = NULL;
        if (choose_backend() < 0)
            return -1;
        Py_BEGIN_ALLOW_THREADS
        st = atg_flac_encode_frames(g_eng, &s->o, s->pcm, fmt, frames, s->sizes, s->n_sizes,
                                    s->channels, s->bps, s->rate, s->frame_no, s->out,
                                    s->out_cap, &nb, s->frame_bytes);
        Py_END_ALLOW_THREADS
    }
    Py_BEGIN_ALLOW_THREADS
    if (st == ATG_OK && nb && fwrite(s->out, 1, nb, s->f) != nb)
        st = (atg_status)1; /* write error, below */
    Py_END_ALLOW_THREADS
    if (st == (atg_status)1) {
        PyErr_SetFromErrno(PyExc_IOError);
        return -1;
    }
    if (st != ATG_OK) {
        if (svc_err) {
            PyErr_SetString(st == ATG_ERR_INVALID || st == ATG_ERR_UNSUPPORTED
                                ? PyExc_ValueError : PyExc_RuntimeError, svc_err);
        } else {
            raise_atg(st);
        }
        return -1;
    }
    for (unsigned i = 0; i < s->n_sizes; ++i) {
        PyObject *t = Py_BuildValue("(KI)", (unsigned long long)s->offset, s->sizes[i]);
        if (!t || PyList_Append(s->list, t) < 0) {
            Py_XDECREF(t);
            return -1;
        }
        Py_DECREF(t);
        s->offset += s->frame_bytes[i];
        if (s->frame_bytes[i] < s->min_fs)
            s->min_fs = s->frame_bytes[i];
        if (s->frame_bytes[i] > s->max_fs)
            s->max_fs = s->frame_bytes[i];
    }
    s->frame_no += s->n_sizes;
    s->n_sizes = 0;
    s->pcm_len = 0;
    return 0;
}

/* one read's FrameList: its samples appended to the segment */
static int take_framelist(enc_state *s, PyObject *fl, uint64_t *frames_out)
{
    PyObject *samples = PyObject_GetAttrString(fl, "samples");
    if (!samples)
        return -1;
    Py_buffer b;
    if (PyObject_GetBuffer(samples, &b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) {
        Py_DECREF(samples);
        return -1;
    }
    int rc = -1;
    if (b.itemsize != 4) {
        PyErr_SetString(PyExc_TypeError, "FrameList samples must be 32-bit integers");
        goto done;
    }
    const int32_t *x = (const int32_t *)b.buf;
    const size_t n = (size_t)(b.len / 4);
    if (n % s->channels) {
        PyErr_SetString(PyExc_ValueError, "FrameList channel count does not match pcmreader");
        goto done;
    }
    *frames_out = n / s->channels;
    const size_t elem = s->bps <= 16 ? 2 : 4;
    if (s->pcm_len + n * elem > s->pcm_cap) {
        size_t cap = s->pcm_cap ? s->pcm_cap : (1u << 20);
        while (cap < s->pcm_len + n * elem)
            cap *= 2;
        uint8_t *p = (uint8_t *)PyMem_Realloc(s->pcm, cap);
        if (!p) {
            PyErr_NoMemory();
            goto done;
        }
        s->pcm = p;
        s->pcm_cap = cap;
    }
    if (elem == 2) {
        int16_t *d = (int16_t *)(s->pcm + s->pcm_len);
        for (size_t i = 0; i < n; ++i)
            d[i] = (int16_t)x[i];
    } else {
        memcpy(s->pcm + s->pcm_len, x, n * 4);
    }
    s->pcm_len += n * elem;
    rc = 0;
done:
    PyBuffer_Release(&b);
    Py_DECREF(samples);
    return rc;
}

static PyObject *encode_flac(PyObject *self, PyObject *args, PyObject *kw)
{
    (void)self;
    static char *kwlist[] = {"filename", "pcmreader", "block_size", "max_lpc_order",
                             "min_residual_partition_order", "max_residual_partition_order",
                             "mid_side", "adaptive_mid_side", "exhaustive_model_search",
                             "disable_verbatim_subframes", "disable_constant_subframes",
                             "disable_fixed_subframes", "disable_lpc_subframes", "padding_size",
                             NULL};
    const char *filename;
    PyObject *reader;
    enc_state s;
    memset(&s, 0, sizeof(s));
    s.o.padding_size = 4096;
    if (!PyArg_ParseTupleAndKeywords(args, kw, "sOIIII|iiiiiiiI", kwlist, &filename, &reader,
                                     &s.o.block_size, &s.o.max_lpc_order,
                                     &s.o.min_residual_partition_order,
                                     &s.o.max_residual_partition_order, &s.o.mid_side,
                                     &s.o.adaptive_mid_side, &s.o.exhaustive_model_search,
                                     &s.o.disable_verbatim_subframes,
                                     &s.o.disable_constant_subframes,
                                     &s.o.disable_fixed_subframes, &s.o.disable_lpc_subframes,
                                     &s.o.padding_size))
        return NULL;
    /* the reader's stream parameters (pcmconv.c:150-196) */
    long v[3];
    static const char *attr[3] = {"channels", "bits_per_sample", "sample_rate"};
    for (int i = 0; i < 3; ++i) {
        PyObject *a = PyObject_GetAttrString(reader, attr[i]);
        if (!a)
            return NULL;
        v[i] = PyLong_AsLong(a);
        Py_DECREF(a);
        if (v[i] == -1 && PyErr_Occurred())
            return NULL;
    }
    if (v[0] < 1 || v[0] > 8 || v[1] < 4 || v[1] > 24 || v[2] < 1) {
        PyErr_SetString(PyExc_ValueError, "unsupported channels / bits_per_sample / sample_rate");
        return NULL;
    }
    s.channels = (unsigned)v[0];
    s.bps = (unsigned)v[1];
    s.rate = (unsigned)v[2];
    s.min_fs = 0xFFFFFFu;
    s.f = fopen(filename, "wb");
    if (!s.f)
        return PyErr_SetFromErrnoWithFilename(PyExc_IOError, filename);
    PyObject *result = NULL;
    uint8_t *hbuf = (uint8_t *)PyMem_Malloc((size_t)s.o.padding_size + 256);
    const uint8_t zero_md5[16] = {0};
    md5_init(&s.md5);
    s.list = PyList_New(0);
    s.frame_bytes = (uint32_t *)PyMem_Malloc(sizeof(uint32_t) * SEGMENT_FRAMES);
    if (!hbuf || !s.list || !s.frame_bytes) {
        PyErr_NoMemory();
        goto fail;
    }
    {
        const uint64_t hn = atg_flac_stream_header(&s.o, s.channels, s.bps, s.rate, 0, 0xFFFFFFu,
                                                   0, zero_md5, hbuf, s.o.padding_size + 256);
        if (!hn) {
            PyErr_SetString(PyExc_ValueError, "invalid padding_size");
            goto fail;
        }
        if (fwrite(hbuf, 1, hn, s.f) != hn) {
            PyErr_SetFromErrnoWithFilename(PyExc_IOError, filename);
            goto fail;
        }
    }
    for (;;) {
        PyObject *fl = PyObject_CallMethod(reader, "read", "I", s.o.block_size);
        if (!fl)
            goto fail; /* the reader's exception propagates (flac.c:244-245) */
        const int ok = PyObject_IsInstance(fl, g_framelist_type);
        if (ok != 1) {
            Py_DECREF(fl);
            if (ok == 0)
                PyErr_SetString(PyExc_TypeError, "results from pcmreader.read() must be FrameLists");
            goto fail;
        }
        uint64_t frames = 0;
        const int r = take_framelist(&s, fl, &frames);
        Py_DECREF(fl);
        if (r < 0)
            goto fail;
        if (!frames)
            break;
        s.sizes[s.n_sizes++] = (uint32_t)frames;
        s.total += frames;
        if (s.n_sizes >= g_segment_frames && flush_segment(&s) < 0)
            goto fail;
    }
    if (flush_segment(&s) < 0)
        goto fail;
    {
        uint8_t digest[16];
        md5_final(&s.md5, digest);
        const uint64_t hn = atg_flac_stream_header(&s.o, s.channels, s.bps, s.rate, s.total,
                                                   s.min_fs, s.max_fs, digest, hbuf,
                                                   s.o.padding_size + 256);
        if (fseek(s.f, 0, SEEK_SET) != 0 || fwrite(hbuf, 1, hn, s.f) != hn) {
            PyErr_SetFromErrnoWithFilename(PyExc_IOError, filename);
            goto fail;
        }
    }
    if (fclose(s.f) != 0) {
        s.f = NULL;
        PyErr_SetFromErrnoWithFilename(PyExc_IOError, filename);
        goto fail;
    }
    s.f = NULL;
    {
        PyObject *c = PyObject_CallMethod(reader, "close", NULL); /* flac.c:282 */
        if (!c)
            goto fail;
        Py_DECREF(c);
    }
    result = s.list;
    s.list = NULL;
fail:
    if (s.f)
        fclose(s.f);
    Py_XDECREF(s.list);
    PyMem_Free(s.pcm);
    PyMem_Free(s.out);
    PyMem_Free(s.frame_bytes);
    PyMem_Free(hbuf);
    return result;
}

/* test hook: frames per GPU call (1..SEGMENT_FRAMES), to exercise
   segment boundaries on short streams */
static PyObject *set_segment_frames(PyObject *self, PyObject *arg)
{
    (void)self;
    const long n = PyLong_AsLong(arg);
    if (n == -1 && PyErr_Occurred())
        return NULL;
    if (n < 1 || n > SEGMENT_FRAMES) {
        PyErr_SetString(PyExc_ValueError, "segment frames must be 1..256");
        return NULL;
    }
    const long old = (long)g_segment_frames;
    g_segment_frames = (unsigned)n;
    return PyLong_FromLong(old);
}

/* gather_into(dst, parts, offset=0) -> bytes written: the parts (objects
   with the buffer protocol, e.g. the int32 sample arrays of a title's
   FrameList reads) copied back to back into the writable buffer dst from
   byte `offset` on, by host threads with the GIL released
   (atg_host_gather) -- album_scan's upload staging (replaygain.py) */
static PyObject *gather_into(PyObject *self, PyObject *args)
{
    (void)self;
    PyObject *dst_o, *parts_o;
    unsigned long long offset = 0;
    if (!PyArg_ParseTuple(args, "OO|K", &dst_o, &parts_o, &offset))
        return NULL;
    PyObject *seq = PySequence_Fast(parts_o, "parts must be a sequence");
    if (!seq)
        return NULL;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    Py_buffer dst;
    if (PyObject_GetBuffer(dst_o, &dst, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0) {
        Py_DECREF(seq);
        return NULL;
    }
    Py_buffer *views = (Py_buffer *)PyMem_Calloc((size_t)(n ? n : 1), sizeof(Py_buffer));
    const void **srcs = (const void **)PyMem_Calloc((size_t)(n ? n : 1), sizeof(void *));
    uint64_t *bytes = (uint64_t *)PyMem_Calloc((size_t)(n ? n : 1), sizeof(uint64_t));
    Py_ssize_t got = 0;
    unsigned long long total = 0;
    PyObject *ret = NULL;
    if (!views || !srcs || !bytes) {
        PyErr_NoMemory();
        goto done;
    }
    for (; got < n; ++got) {
        if (PyObject_GetBuffer(PySequence_Fast_GET_ITEM(seq, got), &views[got],
                               PyBUF_C_CONTIGUOUS) < 0)
            goto done;
        srcs[got] = views[got].buf;
        bytes[got] = (uint64_t)views[got].len;
        total += (unsigned long long)views[got].len;
    }
    if (offset > (unsigned long long)dst.len || total > (unsigned long long)dst.len - offset) {
        PyErr_SetString(PyExc_ValueError, "parts do not fit the destination");
        goto done;
    }
    {
        atg_status st;
        Py_BEGIN_ALLOW_THREADS
        st = atg_host_gather((uint8_t *)dst.buf + offset, srcs, bytes, (uint64_t)n, 0);
        Py_END_ALLOW_THREADS
        if (st != ATG_OK) {
            raise_atg(st);
            goto done;
        }
    }
    ret = PyLong_FromUnsignedLongLong(total);
done:
    for (Py_ssize_t i = 0; i < got; ++i)
        PyBuffer_Release(&views[i]);
    PyMem_Free(views);
    PyMem_Free(srcs);
    PyMem_Free(bytes);
    PyBuffer_Release(&dst);
    Py_DECREF(seq);
    return ret;
}

static PyMethodDef methods[] = {
    {"gather_into", gather_into, METH_VARARGS,
     "gather_into(dst, parts, offset=0) -> bytes: the parts' bytes back to back into dst "
     "(host threads, GIL released)"},
    {"encode_flac", (PyCFunction)(void (*)(void))encode_flac, METH_VARARGS | METH_KEYWORDS,
     "encode_flac(filename, pcmreader, block_size, max_lpc_order, "
     "min_residual_partition_order, max_residual_partition_order, ...) -> "
     "[(byte_offset, pcm_frames), ...]  (FLAC encode on the MI355X)"},
    {"_set_segment_frames", set_segment_frames, METH_O,
     "_set_segment_frames(n) -> previous: FLAC frames per GPU call (test hook)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_encoders_c",
                                    "audiotools encoders on libatgpu (C extension)", -1,
                                    methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__encoders_c(void)
{
    PyObject *pcm = PyImport_ImportModule("audiotools.pcm");
    if (!pcm)
        return NULL;
    g_framelist_type = PyObject_GetAttrString(pcm, "FrameList");
    Py_DECREF(pcm);
    if (!g_framelist_type)
        return NULL;
    return PyModule_Create(&module);
}
