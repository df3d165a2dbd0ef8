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
 * The stream is decoded on the GPU in one batch call (atg_flac_decode_host,
 * flac_decode.hip) the first time a frame is needed after init or a seek;
 * read() then hands out the decoded frames in order and raises the decode
 * status at the frame where the reference's read() would.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <stdint.h>
#include <string.h>

#include "../../../include/atgpu.h"

static PyObject *g_framelist_wrap; /* audiotools.pcm.FrameList._wrap */
static PyObject *g_frombuffer;     /* numpy.frombuffer */
static PyObject *g_int32;          /* numpy.int32 */
static atg_decoder *g_dec;

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
    /* position: byte offset from the first frame, samples left there */
    uint64_t start_byte, remaining;
    int validate, decoded, finalized, closed;
    /* the decode */
    int32_t *pcm;
    uint64_t *starts;      /* PCM frame index of each walked frame, + end */
    uint64_t *offsets;
    uint32_t *block_sizes;
    uint64_t n_walk, n_read, next;
    int status, walk_status;
} FlacDecoderC;

static void drop_decode(FlacDecoderC *self)
{
    PyMem_Free(self->pcm);
    PyMem_Free(self->starts);
    PyMem_Free(self->offsets);
    PyMem_Free(self->block_sizes);
    self->pcm = NULL;
    self->starts = NULL;
    self->offsets = NULL;
    self->block_sizes = NULL;
    self->decoded = 0;
    self->finalized = 0;
    self->next = 0;
}

static void FlacDecoderC_dealloc(FlacDecoderC *self)
{
    drop_decode(self);
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
    drop_decode(self);
    self->closed = 0;
    return 0;
}

/* the GPU decode of the stream from the current position */
static int decode(FlacDecoderC *self)
{
    if (self->decoded)
        return 0;
    if (!g_dec) {
        const char *v = getenv("ATG_DEVICE");
        if (!v)
            v = getenv("LOCAL_RANK");
        if (atg_decoder_create(v ? atoi(v) : 0, &g_dec) != ATG_OK) {
            PyErr_SetString(PyExc_RuntimeError, atg_decoder_last_error());
            return -1;
        }
    }
    const uint8_t *body = (const uint8_t *)PyBytes_AS_STRING(self->data) + self->si.frames_offset;
    const uint64_t blen = (uint64_t)PyBytes_GET_SIZE(self->data) - self->si.frames_offset;
    atg_flac_dec_track t;
    memset(&t, 0, sizeof(t));
    t.data_offset = self->start_byte;
    t.data_bytes = blen - self->start_byte;
    t.total_samples = self->remaining;
    t.sample_rate = self->si.sample_rate;
    t.channels = self->si.channels;
    t.bits_per_sample = self->si.bits_per_sample;
    t.max_block_size = self->si.max_block_size;
    if (self->validate) /* a blank MD5 always verifies (flac.c:488) */
        memcpy(t.md5, self->si.md5, 16);
    atg_flac_dec_result r;
    uint64_t ns = 0, nf = 0;
    atg_status st;
    Py_BEGIN_ALLOW_THREADS
    st = atg_flac_decode_host(g_dec, body, blen, &t, 1, &r, &ns, &nf);
    Py_END_ALLOW_THREADS
    if (st != ATG_OK) {
        PyErr_SetString(PyExc_RuntimeError, atg_decoder_last_error());
        return -1;
    }
    self->pcm = (int32_t *)PyMem_Malloc(sizeof(int32_t) * (ns ? ns : 1));
    self->offsets = (uint64_t *)PyMem_Malloc(sizeof(uint64_t) * (nf ? nf : 1));
    self->block_sizes = (uint32_t *)PyMem_Malloc(sizeof(uint32_t) * (nf ? nf : 1));
    self->starts = (uint64_t *)PyMem_Malloc(sizeof(uint64_t) * (nf + 1));
    if (!self->pcm || !self->offsets || !self->block_sizes || !self->starts) {
        PyErr_NoMemory();
        return -1;
    }
    Py_BEGIN_ALLOW_THREADS
    st = atg_flac_decode_fetch(g_dec, self->pcm, ns, self->offsets, self->block_sizes, nf);
    Py_END_ALLOW_THREADS
    if (st != ATG_OK) {
        PyErr_SetString(PyExc_RuntimeError, atg_decoder_last_error());
        return -1;
    }
    /* PCM frames of each walked frame: MIN(block size, remaining) */
    uint64_t rem = self->remaining, pos = 0;
    self->n_walk = r.walk_frames;
    self->starts[0] = 0;
    for (uint64_t i = 0; i < r.walk_frames; ++i) {
        const uint64_t bs = self->block_sizes[r.first_frame + i];
        pos += bs < rem ? bs : rem;
        rem -= bs;
        self->starts[i + 1] = pos;
    }
    /* frame arrays from the track's first frame */
    if (r.first_frame) {
        memmove(self->offsets, self->offsets + r.first_frame, sizeof(uint64_t) * r.walk_frames);
        memmove(self->block_sizes, self->block_sizes + r.first_frame,
                sizeof(uint32_t) * r.walk_frames);
    }
    if (r.pcm_offset)
        memmove(self->pcm, self->pcm + r.pcm_offset * self->channels,
                sizeof(int32_t) * pos * self->channels);
    self->n_read = r.n_frames;
    self->status = r.status;
    self->walk_status = r.walk_status;
    self->next = 0;
    self->decoded = 1;
    return 0;
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
    if (decode(self) < 0)
        return NULL;
    if (self->next < self->n_read) {
        const uint64_t k = self->next++;
        return framelist(self, self->pcm + self->starts[k] * self->channels,
                         (self->starts[k + 1] - self->starts[k]) * self->channels);
    }
    if (self->status == ATG_FD_OK || self->status == ATG_FD_MD5) {
        self->finalized = 1;
        if (self->status == ATG_FD_MD5)
            return status_error(ATG_FD_MD5);
        return framelist(self, NULL, 0);
    }
    return status_error(self->status);
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
    drop_decode(self);
    return PyLong_FromUnsignedLongLong(sample);
}

static PyObject *FlacDecoderC_offsets(FlacDecoderC *self, PyObject *unused)
{
    (void)unused;
    if (decode(self) < 0)
        return NULL;
    if (self->walk_status != ATG_FD_OK)
        return status_error(self->walk_status);
    self->finalized = 1;
    PyObject *list = PyList_New(0);
    if (!list || self->next >= self->n_walk)
        return list;
    const uint64_t base = self->offsets[self->next];
    for (uint64_t i = self->next; i < self->n_walk; ++i) {
        PyObject *t = Py_BuildValue("(KI)", (unsigned long long)(self->offsets[i] - base),
                                    self->block_sizes[i]);
        if (!t || PyList_Append(list, t) < 0) {
            Py_XDECREF(t);
            Py_DECREF(list);
            return NULL;
        }
        Py_DECREF(t);
    }
    self->next = self->n_walk;
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

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_decoders_c",
                                    "audiotools decoders on libatgpu (C extension)", -1, NULL,
                                    NULL, NULL, NULL, NULL};

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
