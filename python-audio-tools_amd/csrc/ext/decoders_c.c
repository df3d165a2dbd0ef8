/*
 * decoders_c.c — audiotools._decoders_c.FlacDecoder: the reference's
 * CPython decoder type (src/decoders/flac.h:84-108, methods :145-166;
 * src/decoders/flac.c:28-98, 174-443), compiled, over libatgpu's C ABI.
 *
 *   FlacDecoder(file)   a filename or a file object positioned at "fLaC";
 *                       ValueError "not a FLAC file" / IOError "EOF while
 *                       reading metadata" (flacdec_read_metadata,
 *                       flac.c:568-707)
 *   .sample_rate .bits_per_sample .channels .channel_mask
 *   .read(n)            one FLAC frame per call as a pcm.FrameList; after the
 *                       last frame the STREAMINFO MD5 verdict (flac.c:479-493)
 *                       and then empty FrameLists; the reference's ValueError /
 *                       IOError at a bad frame (flac.c:174-285)
 *   .seek(n)            last SEEKTABLE point at or before n (flac.c:287-356)
 *   .offsets()          [(byte offset from the current frame, block size)]
 *                       of the frames left, CRC-16 unchecked (flac.c:365-443)
 *   .close()            later reads / seeks raise ValueError
 *
 * The stream is decoded on the GPU (atg_flac_decode_host, flac_decode.hip)
 * in bounded segments as read() needs them: each call decodes the frames of
 * a window of g_segment_bytes compressed bytes (8 MiB; the decoded PCM held
 * on the host stays ~4x that for 16-bit audio, whatever the stream's
 * length).  A window that ends inside a frame resumes at that frame (the
 * byte the decode reports as walk_end); an error is raised only when the
 * frame that stopped a walk is the first of its window, so it cannot be the
 * window's cut.  read() hands the frames out in order and raises the decode
 * status at the frame where the reference's read() would; the STREAMINFO
 * MD5 is chained over the handed-out frames on the host.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <stdint.h>
#include <string.h>

#include "../../../include/atgpu.h"
#include "md5_host.h"

static PyObject *g_framelist_wrap; /* audiotools.pcm.FrameList._wrap */
static PyObject *g_frombuffer;     /* numpy.frombuffer */
static PyObject *g_int32;          /* numpy.int32 */
static atg_decoder *g_dec;
static uint64_t g_segment_bytes = 8u << 20; /* compressed bytes per GPU call */

static const char *k_msgs[17] = {
    "", "Error", "invalid sync code", "invalid reserved bit", "invalid bits per sample",
    "invalid sample rate", "invalid checksum in frame header",
    "frame sample rate does not match STREAMINFO sample rate",
    "frame channel count does not match STREAMINFO channel count",
    "frame bits-per-sample does not match STREAMINFO bits per sample",
    "frame block size exceeds STREAMINFO's maximum block size",
    "invalid residual partition coding method", "invalid FIXED subframe order",
    "invalid subframe type", "invalid checksum in frame", "EOF reading frame",
    "MD5 mismatch at end of stream"};

static PyObject *status_error(int status)
{
    const char *m = status >= 0 && status <= 16 ? k_msgs[status] : "Error";
    PyErr_SetString(status == ATG_FD_EOF ? PyExc_IOError : PyExc_ValueError, m);
    return NULL;
}

typedef struct {
    PyObject_HEAD
    int sample_rate, bits_per_sample, channels, channel_mask;
    PyObject *data;        /* bytes: the whole image */
    int seekable;
    atg_flac_streaminfo si;
    atg_flac_seekpoint *points;
    uint32_t n_points;
    /* the position read() starts from: byte offset from the first frame and
       remaining_samples there; MD5 validation only from sample 0
       (FlacDecoder_seek, flac.c:317-352) */
    uint64_t start_byte, remaining;
    int validate, finalized, closed;
    /* the segment state */
    uint64_t seg_byte, seg_remaining; /* the next window's first byte / remaining */
    int have_seg;
    int stop;                /* status after the current segment; -1: resume */
    int32_t *pcm;            /* the segment's frames, interleaved */
    uint64_t *starts;        /* PCM frame index of each frame, + end */
    uint64_t *offs;          /* byte offset of each frame from the first frame */
    uint64_t *rems;          /* remaining_samples at each frame */
    uint64_t seg_n, next;
    uint64_t after_byte, after_rem; /* where the frame after the segment sits */
    int md5_on;
    md5_ctx md5;
    /* scratch of the fetch (grown as needed) */
    uint64_t *f_offs;
    uint32_t *f_bs;
    uint64_t f_cap;
} FlacDecoderC;

static void drop_segment(FlacDecoderC *self)
{
    PyMem_Free(self->pcm);
    PyMem_Free(self->starts);
    PyMem_Free(self->offs);
    PyMem_Free(self->rems);
    self->pcm = NULL;
    self->starts = NULL;
    self->offs = NULL;
    self->rems = NULL;
    self->have_seg = 0;
    self->seg_n = 0;
    self->next = 0;
}

/* back to the position (init, seek): no segment, a fresh MD5 */
static void reset_stream(FlacDecoderC *self)
{
    drop_segment(self);
    self->finalized = 0;
    self->seg_byte = self->start_byte;
    self->seg_remaining = self->remaining;
    self->stop = -1;
    /* FlacDecoder_verify_okay (flac.c:479-493): a blank MD5 always passes */
    int any = 0;
    for (int i = 0; i < 16; ++i)
        any |= self->si.md5[i];
    self->md5_on = self->validate && any;
    md5_init(&self->md5);
}

static void FlacDecoderC_dealloc(FlacDecoderC *self)
{
    drop_segment(self);
    PyMem_Free(self->f_offs);
    PyMem_Free(self->f_bs);
    PyMem_Free(self->points);
    Py_XDECREF(self->data);
    Py_TYPE(self)->tp_free((PyObject *)self);
}

static int FlacDecoderC_init(FlacDecoderC *self, PyObject *args, PyObject *kw)
{
    (void)kw;
    PyObject *file;
    if (!PyArg_ParseTuple(args, "O", &file))
        return -1;
    PyObject *data = NULL;
    if (PyUnicode_Check(file)) {
        PyObject *io = PyImport_ImportModule("io");
        if (!io)
            return -1;
        PyObject *f = PyObject_CallMethod(io, "open", "Os", file, "rb");
        Py_DECREF(io);
        if (!f)
            return -1;
        data = PyObject_CallMethod(f, "read", NULL);
        PyObject *c = PyObject_CallMethod(f, "close", NULL);
        Py_XDECREF(c);
        Py_DECREF(f);
        self->seekable = 1;
    } else if (PyBytes_Check(file)) {
        data = file;
        Py_INCREF(data);
        self->seekable = 0;
    } else if (PyByteArray_Check(file) || PyMemoryView_Check(file)) {
        data = PyBytes_FromObject(file); /* raw bytes cannot seek */
        self->seekable = 0;
    } else {
        data = PyObject_CallMethod(file, "read", NULL);
        self->seekable = 1;
    }
    if (!data)
        return -1;
    if (!PyBytes_Check(data)) {
        Py_DECREF(data);
        PyErr_SetString(PyExc_TypeError, "file.read() must return bytes");
        return -1;
    }
    Py_XSETREF(self->data, data);
    const uint8_t *p = (const uint8_t *)PyBytes_AS_STRING(data);
    const uint64_t len = (uint64_t)PyBytes_GET_SIZE(data);
    int rc = atg_flac_read_metadata(p, len, &self->si, NULL, 0);
    if (rc == 0 && self->si.n_seekpoints) {
        self->points = (atg_flac_seekpoint *)PyMem_Malloc(sizeof(atg_flac_seekpoint) *
                                                          self->si.n_seekpoints);
        if (!self->points) {
            PyErr_NoMemory();
            return -1;
        }
        rc = atg_flac_read_metadata(p, len, &self->si, self->points, self->si.n_seekpoints);
        self->n_points = self->si.n_seekpoints;
    }
    if (rc == 1) {
        PyErr_SetString(PyExc_ValueError, "not a FLAC file");
        return -1;
    }
    if (rc) {
        PyErr_SetString(PyExc_IOError, "EOF while reading metadata");
        return -1;
    }
    self->sample_rate = (int)self->si.sample_rate;
    self->bits_per_sample = (int)self->si.bits_per_sample;
    self->channels = (int)self->si.channels;
    self->channel_mask = (int)self->si.channel_mask;
    self->start_byte = 0;
    self->remaining = self->si.total_samples;
    self->validate = 1;
    reset_stream(self);
    self->closed = 0;
    return 0;
}

static int ensure_decoder(void)
{
    if (g_dec)
        return 0;
    /* ATG_DEVICE, LOCAL_RANK, else the node-wide round robin */
    if (atg_decoder_create(atg_pick_device(), &g_dec) != ATG_OK) {
        PyErr_SetString(PyExc_RuntimeError, atg_decoder_last_error());
        return -1;
    }
    return 0;
}

/* one GPU decode of body[start, end) with `rem` samples left; the PCM (if
   pcm_out) and the frame arrays land in fresh / scratch buffers */
static int decode_window(FlacDecoderC *self, uint64_t start, uint64_t end, uint64_t rem,
                         int want_pcm, atg_flac_dec_result *r, int32_t **pcm_out)
{
    if (ensure_decoder() < 0)
        return -1;
    const uint8_t *body = (const uint8_t *)PyBytes_AS_STRING(self->data) + self->si.frames_offset;
    atg_flac_dec_track t;
    memset(&t, 0, sizeof(t));
    t.data_offset = 0;
    t.data_bytes = end - start;
    t.total_samples = rem;
    t.sample_rate = self->si.sample_rate;
    t.channels = self->si.channels;
    t.bits_per_sample = self->si.bits_per_sample;
    t.max_block_size = self->si.max_block_size;
    /* t.md5 stays blank: the MD5 is chained over the segments on the host */
    uint64_t ns = 0, nf = 0;
    atg_status st;
    Py_BEGIN_ALLOW_THREADS
    st = atg_flac_decode_host(g_dec, body + start, end - start, &t, 1, r, &ns, &nf);
    Py_END_ALLOW_THREADS
    if (st != ATG_OK) {
        PyErr_SetString(PyExc_RuntimeError, atg_decoder_last_error());
        return -1;
    }
    if (nf + 1 > self->f_cap) {
        uint64_t *o = (uint64_t *)PyMem_Realloc(self->f_offs, sizeof(uint64_t) * (nf + 1));
        if (o)
            self->f_offs = o;
        uint32_t *b = (uint32_t *)PyMem_Realloc(self->f_bs, sizeof(uint32_t) * (nf + 1));
        if (b)
            self->f_bs = b;
        if (!o || !b) {
            PyErr_NoMemory();
            return -1;
        }
        self->f_cap = nf + 1;
    }
    int32_t *pcm = NULL;
    if (want_pcm) {
        pcm = (int32_t *)PyMem_Malloc(sizeof(int32_t) * (ns ? ns : 1));
        if (!pcm) {
            PyErr_NoMemory();
            return -1;
        }
    }
    Py_BEGIN_ALLOW_THREADS
    st = atg_flac_decode_fetch(g_dec, pcm, want_pcm ? ns : 0, self->f_offs, self->f_bs, nf);
    Py_END_ALLOW_THREADS
    if (st != ATG_OK) {
        PyMem_Free(pcm);
        PyErr_SetString(PyExc_RuntimeError, atg_decoder_last_error());
        return -1;
    }
    if (pcm_out)
        *pcm_out = pcm;
    return 0;
}

/* decode the next segment from (seg_byte, seg_remaining) */
static int decode_segment(FlacDecoderC *self)
{
    const uint64_t blen = (uint64_t)PyBytes_GET_SIZE(self->data) - self->si.frames_offset;
    const uint64_t start = self->seg_byte;
    uint64_t rem = self->seg_remaining;
    uint64_t win = g_segment_bytes;
    atg_flac_dec_result r;
    int32_t *pcm = NULL;
    int final;
    for (;;) {
        const uint64_t end = start + win < blen && start + win > start ? start + win : blen;
        final = end >= blen;
        if (decode_window(self, start, end, rem, 1, &r, &pcm) < 0)
            return -1;
        if (r.status == ATG_FD_OK || final || r.n_frames > 0 || r.status == ATG_FD_FRAME_CRC)
            break;
        PyMem_Free(pcm); /* the window's first frame is longer than the window */
        pcm = NULL;
        win *= 4;
    }
    drop_segment(self);
    const uint64_t n = r.n_frames;
    self->starts = (uint64_t *)PyMem_Malloc(sizeof(uint64_t) * (n + 1));
    self->offs = (uint64_t *)PyMem_Malloc(sizeof(uint64_t) * (n ? n : 1));
    self->rems = (uint64_t *)PyMem_Malloc(sizeof(uint64_t) * (n ? n : 1));
    if (!self->starts || !self->offs || !self->rems) {
        PyMem_Free(pcm);
        drop_segment(self);
        PyErr_NoMemory();
        return -1;
    }
    /* PCM frames of each frame: MIN(block size, remaining); remaining
       wraps as the reference's uint64 remaining_samples */
    uint64_t pos = 0;
    self->starts[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t bs = self->f_bs[r.first_frame + i];
        self->rems[i] = rem;
        self->offs[i] = start + self->f_offs[r.first_frame + i];
        pos += bs < rem ? bs : rem;
        rem -= bs;
        self->starts[i + 1] = pos;
    }
    self->after_byte = start + (r.walk_frames > n ? self->f_offs[r.first_frame + n] : r.walk_end);
    self->after_rem = rem;
    if (r.pcm_offset)
        memmove(pcm, pcm + r.pcm_offset * self->channels,
                sizeof(int32_t) * pos * self->channels);
    self->pcm = pcm;
    self->seg_n = n;
    self->next = 0;
    self->have_seg = 1;
    if (r.status == ATG_FD_OK)
        self->stop = ATG_FD_OK;          /* remaining_samples reached 0 */
    else if (final || n == 0 || r.status == ATG_FD_FRAME_CRC)
        self->stop = r.status;           /* a real error at frame n */
    else {                               /* the window's cut: resume there */
        self->stop = -1;
        self->seg_byte = start + r.walk_end;
        self->seg_remaining = rem;
    }
    return 0;
}

/* the frame's FrameList.to_bytes(False, True) into the MD5: little-endian,
   saturated to the bps range (src/pcm.c:1826-1948) */
static void md5_frame(FlacDecoderC *self, const int32_t *x, uint64_t n)
{
    const int bps = self->bits_per_sample;
    const unsigned width = (unsigned)(bps + 7) / 8;
    const int64_t hi = ((int64_t)1 << (bps - 1)) - 1, lo = -hi - 1;
    uint8_t tmp[4096];
    size_t tl = 0;
    for (uint64_t i = 0; i < n; ++i) {
        int64_t v = x[i];
        v = v < lo ? lo : v > hi ? hi : v;
        for (unsigned k = 0; k < width; ++k)
            tmp[tl++] = (uint8_t)((uint64_t)v >> (8 * k));
        if (tl + 4 > sizeof(tmp)) {
            md5_update(&self->md5, tmp, tl);
            tl = 0;
        }
    }
    md5_update(&self->md5, tmp, tl);
}

static PyObject *framelist(FlacDecoderC *self, const int32_t *x, uint64_t n_samples)
{
    PyObject *b = PyBytes_FromStringAndSize((const char *)x, (Py_ssize_t)(4 * n_samples));
    if (!b)
        return NULL;
    PyObject *a = PyObject_CallFunctionObjArgs(g_frombuffer, b, g_int32, NULL);
    Py_DECREF(b);
    if (!a)
        return NULL;
    PyObject *fl = PyObject_CallFunction(g_framelist_wrap, "Oii", a, self->channels,
                                         self->bits_per_sample);
    Py_DECREF(a);
    return fl;
}

static PyObject *FlacDecoderC_read(FlacDecoderC *self, PyObject *args)
{
    int n;
    if (!PyArg_ParseTuple(args, "i", &n))
        return NULL;
    if (self->closed) {
        PyErr_SetString(PyExc_ValueError, "cannot read closed stream");
        return NULL;
    }
    if (self->finalized)
        return framelist(self, NULL, 0);
    while (!self->have_seg || self->next >= self->seg_n) {
        if (self->have_seg && self->stop >= 0) {
            /* every good frame handed out: the stream either reached
               remaining_samples == 0 (MD5 verdict) or stops on an error */
            if (self->stop == ATG_FD_OK) {
                self->finalized = 1;
                if (self->md5_on) {
                    uint8_t d[16];
                    md5_final(&self->md5, d);
                    if (memcmp(d, self->si.md5, 16) != 0)
                        return status_error(ATG_FD_MD5);
                }
                return framelist(self, NULL, 0);
            }
            return status_error(self->stop);
        }
        if (decode_segment(self) < 0)
            return NULL;
    }
    const uint64_t k = self->next++;
    const int32_t *x = self->pcm + self->starts[k] * self->channels;
    const uint64_t ns = (self->starts[k + 1] - self->starts[k]) * self->channels;
    if (self->md5_on)
        md5_frame(self, x, ns);
    return framelist(self, x, ns);
}

static PyObject *FlacDecoderC_seek(FlacDecoderC *self, PyObject *args)
{
    long long target;
    if (!PyArg_ParseTuple(args, "L", &target))
        return NULL;
    if (self->closed) {
        PyErr_SetString(PyExc_ValueError, "cannot seek closed stream");
        return NULL;
    }
    if (!self->seekable) {
        PyErr_SetString(PyExc_TypeError, "can only seek streams from file objects");
        return NULL;
    }
    if (target < 0) {
        PyErr_SetString(PyExc_ValueError, "cannot seek to negative value");
        return NULL;
    }
    uint64_t sample = 0, byte = 0;
    for (uint32_t i = 0; i < self->n_points; ++i) {
        if (self->points[i].sample_number <= (uint64_t)target) {
            sample = self->points[i].sample_number;
            byte = self->points[i].byte_offset;
        } else {
            break;
        }
    }
    self->start_byte = byte;
    self->remaining = self->si.total_samples - sample;
    self->validate = sample == 0;
    reset_stream(self);
    return PyLong_FromUnsignedLongLong(sample);
}

static PyObject *FlacDecoderC_offsets(FlacDecoderC *self, PyObject *unused)
{
    (void)unused;
    /* the current position: the next frame read() would hand out */
    uint64_t pos, rem;
    if (self->have_seg && self->next < self->seg_n) {
        pos = self->offs[self->next];
        rem = self->rems[self->next];
    } else if (self->have_seg && self->stop == ATG_FD_OK) {
        self->finalized = 1;
        return PyList_New(0); /* remaining_samples already 0 */
    } else if (self->have_seg) {
        pos = self->after_byte; /* the next window, or the frame that failed */
        rem = self->after_rem;
    } else {
        pos = self->seg_byte;
        rem = self->seg_remaining;
    }
    const uint64_t blen = (uint64_t)PyBytes_GET_SIZE(self->data) - self->si.frames_offset;
    atg_flac_dec_result r;
    if (decode_window(self, pos, blen, rem, 0, &r, NULL) < 0)
        return NULL;
    if (r.walk_status != ATG_FD_OK)
        return status_error(r.walk_status);
    self->finalized = 1;
    PyObject *list = PyList_New(0);
    if (!list)
        return NULL;
    for (uint64_t i = 0; i < r.walk_frames; ++i) {
        PyObject *t = Py_BuildValue("(KI)", (unsigned long long)self->f_offs[r.first_frame + i],
                                    self->f_bs[r.first_frame + i]);
        if (!t || PyList_Append(list, t) < 0) {
            Py_XDECREF(t);
            Py_DECREF(list);
            return NULL;
        }
        Py_DECREF(t);
    }
    return list;
}

static PyObject *FlacDecoderC_close(FlacDecoderC *self, PyObject *unused)
{
    (void)unused;
    self->closed = 1;
    Py_RETURN_NONE;
}

static PyMemberDef members[] = {
    {"sample_rate", T_INT, offsetof(FlacDecoderC, sample_rate), READONLY, "sample rate"},
    {"bits_per_sample", T_INT, offsetof(FlacDecoderC, bits_per_sample), READONLY,
     "bits per sample"},
    {"channels", T_INT, offsetof(FlacDecoderC, channels), READONLY, "channel count"},
    {"channel_mask", T_INT, offsetof(FlacDecoderC, channel_mask), READONLY, "channel mask"},
    {NULL, 0, 0, 0, NULL}};

static PyMethodDef dec_methods[] = {
    {"read", (PyCFunction)FlacDecoderC_read, METH_VARARGS, "read(pcm_frames) -> FrameList"},
    {"seek", (PyCFunction)FlacDecoderC_seek, METH_VARARGS, "seek(pcm_frame_offset) -> int"},
    {"offsets", (PyCFunction)FlacDecoderC_offsets, METH_NOARGS,
     "offsets() -> [(byte offset, block size), ...]"},
    {"close", (PyCFunction)FlacDecoderC_close, METH_NOARGS, "close()"},
    {NULL, NULL, 0, NULL}};

static PyTypeObject FlacDecoderType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "audiotools._decoders_c.FlacDecoder",
    .tp_basicsize = sizeof(FlacDecoderC),
    .tp_dealloc = (destructor)FlacDecoderC_dealloc,
    .tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE,
    .tp_doc = "FLAC decoder on the MI355X (reference audiotools.decoders.FlacDecoder)",
    .tp_methods = dec_methods,
    .tp_members = members,
    .tp_init = (initproc)FlacDecoderC_init,
    .tp_new = PyType_GenericNew,
};

/* test hook: compressed bytes per GPU decode call */
static PyObject *set_segment_bytes(PyObject *self, PyObject *arg)
{
    (void)self;
    const unsigned long long n = PyLong_AsUnsignedLongLong(arg);
    if (n == (unsigned long long)-1 && PyErr_Occurred())
        return NULL;
    if (n < 1) {
        PyErr_SetString(PyExc_ValueError, "segment bytes must be positive");
        return NULL;
    }
    const uint64_t old = g_segment_bytes;
    g_segment_bytes = n;
    return PyLong_FromUnsignedLongLong(old);
}

static PyMethodDef module_methods[] = {
    {"_set_segment_bytes", set_segment_bytes, METH_O,
     "_set_segment_bytes(n) -> previous: compressed bytes per GPU decode call (test hook)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_decoders_c",
                                    "audiotools decoders on libatgpu (C extension)", -1,
                                    module_methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__decoders_c(void)
{
    PyObject *pcm = PyImport_ImportModule("audiotools.pcm");
    if (!pcm)
        return NULL;
    PyObject *fl = PyObject_GetAttrString(pcm, "FrameList");
    Py_DECREF(pcm);
    if (!fl)
        return NULL;
    g_framelist_wrap = PyObject_GetAttrString(fl, "_wrap");
    Py_DECREF(fl);
    PyObject *np = PyImport_ImportModule("numpy");
    if (!g_framelist_wrap || !np)
        return NULL;
    g_frombuffer = PyObject_GetAttrString(np, "frombuffer");
    g_int32 = PyObject_GetAttrString(np, "int32");
    Py_DECREF(np);
    if (!g_frombuffer || !g_int32)
        return NULL;
    if (PyType_Ready(&FlacDecoderType) < 0)
        return NULL;
    PyObject *m = PyModule_Create(&module);
    if (!m)
        return NULL;
    Py_INCREF(&FlacDecoderType);
    if (PyModule_AddObject(m, "FlacDecoder", (PyObject *)&FlacDecoderType) < 0) {
        Py_DECREF(&FlacDecoderType);
        Py_DECREF(m);
        return NULL;
    }
    return m;
}
