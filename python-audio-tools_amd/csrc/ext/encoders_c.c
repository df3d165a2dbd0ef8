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
 * the STREAMINFO MD5 of the PCM bytes is updated per read on the host
 * (RFC 1321 below), as the reference's read callback does
 * (pcmconv.c:266-291).  Host memory stays bounded by one segment.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/atgpu.h"

#define SEGMENT_FRAMES 256

/* ------------------------------------------------------------------ MD5 */
typedef struct {
    uint32_t h[4];
    uint64_t len;
    uint8_t buf[64];
} md5_ctx;

static uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

static void md5_block(uint32_t h[4], const uint8_t *p)
{
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t X[16];
    for (int i = 0; i < 16; ++i)
        X[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) |
               ((uint32_t)p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; ++i) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + rol(a + f + K[i] + X[g], S[i]);
        a = t;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

static void md5_init(md5_ctx *m)
{
    m->h[0] = 0x67452301u;
    m->h[1] = 0xefcdab89u;
    m->h[2] = 0x98badcfeu;
    m->h[3] = 0x10325476u;
    m->len = 0;
}

static void md5_update(md5_ctx *m, const uint8_t *p, size_t n)
{
    size_t have = (size_t)(m->len & 63u);
    m->len += n;
    if (have) {
        const size_t take = 64 - have < n ? 64 - have : n;
        memcpy(m->buf + have, p, take);
        p += take;
        n -= take;
        if (have + take < 64)
            return;
        md5_block(m->h, m->buf);
    }
    for (; n >= 64; p += 64, n -= 64)
        md5_block(m->h, p);
    memcpy(m->buf, p, n);
}

static void md5_final(md5_ctx *m, uint8_t out[16])
{
    const uint64_t bits = m->len * 8u;
    static const uint8_t pad[64] = {0x80};
    const size_t have = (size_t)(m->len & 63u);
    md5_update(m, pad, have < 56 ? 56 - have : 120 - have);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i)
        lb[i] = (uint8_t)(bits >> (8 * i));
    md5_update(m, lb, 8);
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k)
            out[4 * i + k] = (uint8_t)(m->h[i] >> (8 * k));
}

/* ------------------------------------------------------------- module */
static PyObject *g_framelist_type; /* audiotools.pcm.FrameList */
static atg_engine *g_eng;

static int engine_device(void)
{
    const char *v = getenv("ATG_DEVICE");
    if (!v)
        v = getenv("LOCAL_RANK");
    return v ? atoi(v) : 0;
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
} enc_state;

/* encode and write the collected segment; appends to the offsets list */
static int flush_segment(enc_state *s)
{
    if (!s->n_sizes)
        return 0;
    if (!g_eng) {
        const atg_status st = atg_engine_create(engine_device(), &g_eng);
        if (st != ATG_OK) {
            raise_atg(st);
            return -1;
        }
    }
    const size_t elem = s->bps <= 16 ? 2 : 4;
    const uint64_t frames = s->pcm_len / (elem * s->channels);
    const uint64_t cap = atg_flac_max_frames_bytes(&s->o, frames, s->sizes, s->n_sizes,
                                                   s->channels, s->bps);
    if (!cap) {
        PyErr_SetString(PyExc_ValueError, "invalid encoder options");
        return -1;
    }
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
    Py_BEGIN_ALLOW_THREADS
    st = atg_flac_encode_frames(g_eng, &s->o, s->pcm, s->bps <= 16 ? ATG_PCM_S16 : ATG_PCM_S32,
                                frames, s->sizes, s->n_sizes, s->channels, s->bps, s->rate,
                                s->frame_no, s->out, s->out_cap, &nb, s->frame_bytes);
    if (st == ATG_OK && nb && fwrite(s->out, 1, nb, s->f) != nb)
        st = (atg_status)1; /* write error, below */
    Py_END_ALLOW_THREADS
    if (st == (atg_status)1) {
        PyErr_SetFromErrno(PyExc_IOError);
        return -1;
    }
    if (st != ATG_OK) {
        raise_atg(st);
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

/* one read's FrameList: its samples appended to the segment, its PCM
   bytes (little-endian, signed) into the MD5 */
static int take_framelist(enc_state *s, PyObject *fl, md5_ctx *md5, uint64_t *frames_out)
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
    const unsigned width = (s->bps + 7) / 8;
    uint8_t tmp[4096];
    size_t tl = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t v = (uint32_t)x[i];
        if (elem == 2) {
            const int16_t h = (int16_t)x[i];
            memcpy(s->pcm + s->pcm_len + 2 * i, &h, 2);
        } else {
            memcpy(s->pcm + s->pcm_len + 4 * i, &x[i], 4);
        }
        for (unsigned k = 0; k < width; ++k)
            tmp[tl++] = (uint8_t)(v >> (8 * k));
        if (tl + 4 > sizeof(tmp)) {
            md5_update(md5, tmp, tl);
            tl = 0;
        }
    }
    md5_update(md5, tmp, tl);
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
    md5_ctx md5;
    md5_init(&md5);
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
        const int r = take_framelist(&s, fl, &md5, &frames);
        Py_DECREF(fl);
        if (r < 0)
            goto fail;
        if (!frames)
            break;
        s.sizes[s.n_sizes++] = (uint32_t)frames;
        s.total += frames;
        if (s.n_sizes == SEGMENT_FRAMES && flush_segment(&s) < 0)
            goto fail;
    }
    if (flush_segment(&s) < 0)
        goto fail;
    {
        uint8_t digest[16];
        md5_final(&md5, digest);
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

static PyMethodDef methods[] = {
    {"encode_flac", (PyCFunction)(void (*)(void))encode_flac, METH_VARARGS | METH_KEYWORDS,
     "encode_flac(filename, pcmreader, block_size, max_lpc_order, "
     "min_residual_partition_order, max_residual_partition_order, ...) -> "
     "[(byte_offset, pcm_frames), ...]  (FLAC encode on the MI355X)"},
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
