/*
 * aioquic_amd._crypto -- CPython binding of libquicpp.so (include/quic_pp.h).
 *
 * Built like the reference's aioquic._crypto: limited API 3.10 (abi3) and
 * heap types from PyType_FromSpec (src/aioquic/_crypto.c:203-219,358-372,
 * setup.py:30-39), so one binary serves every CPython >= 3.10.
 *
 * Object API identical to the reference (src/aioquic/_crypto.pyi:1-15):
 *   AEAD(cipher_name, key, iv).encrypt(data, associated_data, packet_number) -> bytes
 *                             .decrypt(data, associated_data, packet_number) -> bytes
 *   HeaderProtection(cipher_name, key).apply(plain_header, protected_payload) -> bytes
 *                                     .remove(packet, encrypted_offset) -> (bytes, int)
 *   CryptoError(ValueError), with the reference's messages (_crypto.c:17-29,79-90,126-152).
 * Every byte of crypto runs on the GPU through libquicpp; there is no CPU path.
 * Without a gfx950 device the constructors raise RuntimeError.
 *
 * Batch API (pointers are ints: device pointers for the device forms, host
 * pointers for the *_into forms; the caller keeps the memory alive):
 *   KeyTable(capacity) .set(materials) .derive(secrets) .clear(slots) .capacity
 *   Plan(capacity)                                  device scratch of the bucketing step
 *   protect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream[, plan])   -> None
 *   unprotect(...)                                                          -> None
 *   plan_build(plan, table, desc_ptr, n, stream)    bucket a batch by (suite, slot)
 *   protect_host(table, desc, data, out_len) -> (bytes out, bytes results)
 *   unprotect_host(table, desc, data, out_len) -> (bytes out, bytes results)
 *   protect_into(table, desc_ptr, n, in_ptr, in_len, out_ptr, out_len, res_ptr) -> None
 *   unprotect_into(...)                                                         -> None
 *   hp_mask_host(table, slots, samples) -> bytes
 *   protect_datagrams(...), unprotect_walk(...)     the batched callers' C paths
 *   MultiSession(devices, key_capacity)             one host batch over several GPUs
 *
 * Threads: host-buffer calls release the GIL.  Each OS thread gets its own
 * qpp_session (pinned staging + streams; quic_pp.h: a session is single-
 * threaded), created on first use and destroyed when the thread exits, so
 * concurrent calls from different threads never share staging.
 */
#define PY_SSIZE_T_CLEAN
#define Py_LIMITED_API 0x030A0000
#include <Python.h>
#include <ctype.h>
#include <pthread.h>
#include <string.h>

#include "quic_pp.h"

static PyObject *g_crypto_error;
static PyObject *g_aead_type, *g_hp_type, *g_kt_type, *g_plan_type, *g_multi_type;

/* ------------------------------------------------------------ sessions -- */

static pthread_key_t g_session_key;
static pthread_once_t g_session_once = PTHREAD_ONCE_INIT;

static void session_free(void *s) { qpp_session_destroy((qpp_session *)s); }
static void session_key_init(void) { (void)pthread_key_create(&g_session_key, session_free); }

/* This thread's session, created on first use.  Call with the GIL held. */
static qpp_session *session(void)
{
    (void)pthread_once(&g_session_once, session_key_init);
    qpp_session *s = (qpp_session *)pthread_getspecific(g_session_key);
    if (s) return s;
    int rc = qpp_session_create(1 << 16, 64, &s);
    if (rc != QPP_OK) {
        PyErr_Format(PyExc_RuntimeError, "aioquic_amd: cannot open a gfx950 session (%s)",
                     qpp_strerror(rc));
        return NULL;
    }
    if (pthread_setspecific(g_session_key, s) != 0) {
        qpp_session_destroy(s);
        PyErr_SetString(PyExc_RuntimeError, "aioquic_amd: cannot store the thread's session");
        return NULL;
    }
    return s;
}

static int check_rc(int rc)
{
    if (rc == QPP_OK) return 0;
    PyErr_Format(PyExc_RuntimeError, "aioquic_amd: %s", qpp_strerror(rc));
    return -1;
}

static void *as_ptr(unsigned long long v) { return (void *)(uintptr_t)v; }

static void heap_dealloc(PyObject *self)
{
    PyTypeObject *tp = Py_TYPE(self);
    freefunc f = (freefunc)PyType_GetSlot(tp, Py_tp_free);
    f(self);
    Py_DECREF(tp);
}

/* --------------------------------------------------------- cipher names -- */

static int streq_ci(const char *a, Py_ssize_t alen, const char *b)
{
    if ((size_t)alen != strlen(b)) return 0;
    for (Py_ssize_t i = 0; i < alen; ++i)
        if (tolower((unsigned char)a[i]) != b[i]) return 0;
    return 1;
}

/* EVP cipher names the reference maps to each suite (quic/crypto.py:12-16) */
static int aead_suite(const char *name, Py_ssize_t len)
{
    if (streq_ci(name, len, "aes-128-gcm") || streq_ci(name, len, "id-aes128-gcm")) return QPP_AES_128_GCM;
    if (streq_ci(name, len, "aes-256-gcm") || streq_ci(name, len, "id-aes256-gcm")) return QPP_AES_256_GCM;
    if (streq_ci(name, len, "chacha20-poly1305")) return QPP_CHACHA20_POLY1305;
    return -1;
}

static int hp_suite(const char *name, Py_ssize_t len)
{
    if (streq_ci(name, len, "aes-128-ecb")) return QPP_AES_128_GCM;
    if (streq_ci(name, len, "aes-256-ecb")) return QPP_AES_256_GCM;
    if (streq_ci(name, len, "chacha20")) return QPP_CHACHA20_POLY1305;
    return -1;
}

static int suite_key_len(int suite) { return suite == QPP_AES_128_GCM ? 16 : 32; }

/* --------------------------------------------------- parallel host copy -- */

/* Many (dst, src, len) copies between caller memory and pinned staging, split
 * over up to 8 threads by bytes (one thread streams ~6-10 GB/s, well under
 * the PCIe rate).  Small totals stay on the calling thread.  Call without the
 * GIL only when every buffer is kept alive by the caller. */
typedef struct {
    uint8_t **dst;
    const uint8_t **src;
    const size_t *len;
    size_t b, e;
} CopyJob;

static void *copy_job(void *arg)
{
    CopyJob *j = (CopyJob *)arg;
    for (size_t i = j->b; i < j->e; ++i) memcpy(j->dst[i], j->src[i], j->len[i]);
    return NULL;
}

static void par_copy(uint8_t **dst, const uint8_t **src, const size_t *len, size_t n, size_t total)
{
    enum { kThreads = 8 };
    const size_t kMin = (size_t)4 << 20;
    int parts = total >= kMin ? (int)(total / (kMin / 2)) : 1;
    if (parts > kThreads) parts = kThreads;
    if (parts < 2 || n < 2) {
        CopyJob j = {dst, src, len, 0, n};
        copy_job(&j);
        return;
    }
    CopyJob jobs[kThreads];
    pthread_t th[kThreads];
    int started[kThreads] = {0};
    size_t i = 0, acc = 0;
    for (int t = 0; t < parts; ++t) {
        const size_t goal = total / parts * (size_t)(t + 1);
        jobs[t].dst = dst;
        jobs[t].src = src;
        jobs[t].len = len;
        jobs[t].b = i;
        while (i < n && (acc < goal || t == parts - 1)) acc += len[i++];
        jobs[t].e = i;
    }
    for (int t = 1; t < parts; ++t) started[t] = pthread_create(&th[t], NULL, copy_job, &jobs[t]) == 0;
    copy_job(&jobs[0]);
    for (int t = 1; t < parts; ++t) {
        if (started[t]) pthread_join(th[t], NULL);
        else copy_job(&jobs[t]);
    }
}

/* ------------------------------------------------------------ key slot -- */

/* A single-slot device key table, created on first use.  The slot is
 * read-only after creation, so objects may be used from any thread. */
typedef struct {
    qpp_key_material km;
    qpp_keytab *kt;
} OneSlot;

static int oneslot_ready(OneSlot *o)
{
    if (o->kt) return 0;
    qpp_session *s = session();
    if (!s) return -1;
    int rc = qpp_keytab_create(1, &o->kt);
    if (rc == QPP_OK) rc = qpp_session_set_keys(s, o->kt, &o->km, 1);
    if (rc != QPP_OK) {
        if (o->kt) qpp_keytab_destroy(o->kt);
        o->kt = NULL;
        return check_rc(rc);
    }
    return 0;
}

static void oneslot_reset(OneSlot *o, int suite)
{
    if (o->kt) qpp_keytab_destroy(o->kt);
    o->kt = NULL;
    memset(&o->km, 0, sizeof(o->km));
    o->km.suite = (uint8_t)suite;
}

/* ---------------------------------------------------------------- AEAD -- */

typedef struct {
    PyObject_HEAD
    OneSlot s;
} AEADObject;

static int AEAD_init(AEADObject *self, PyObject *args, PyObject *kwargs)
{
    const char *name;
    const unsigned char *key, *iv;
    Py_ssize_t name_len, key_len, iv_len;
    if (!PyArg_ParseTuple(args, "y#y#y#", &name, &name_len, &key, &key_len, &iv, &iv_len))
        return -1;
    int suite = aead_suite(name, name_len);
    if (suite < 0) {
        PyErr_Format(g_crypto_error, "Invalid cipher name: %s", name);
        return -1;
    }
    if (key_len > 32) {
        PyErr_SetString(g_crypto_error, "Invalid key length");
        return -1;
    }
    if (iv_len > 12) {
        PyErr_SetString(g_crypto_error, "Invalid iv length");
        return -1;
    }
    if (key_len != suite_key_len(suite)) {
        /* the reference fails in EVP_CIPHER_CTX_set_key_length */
        PyErr_SetString(g_crypto_error, "OpenSSL call failed");
        return -1;
    }
    oneslot_reset(&self->s, suite);
    memcpy(self->s.km.key, key, (size_t)key_len);
    memcpy(self->s.km.iv, iv, (size_t)iv_len); /* short iv: zero padded, as the reference */
    return oneslot_ready(&self->s);
}

static void AEAD_dealloc(AEADObject *self)
{
    if (self->s.kt) qpp_keytab_destroy(self->s.kt);
    heap_dealloc((PyObject *)self);
}

/* in = aad || data; AEAD only (QPP_F_NO_HP) */
static PyObject *aead_run(AEADObject *self, PyObject *args, int enc)
{
    const unsigned char *data, *aad;
    Py_ssize_t data_len, aad_len;
    unsigned long long pn;
    if (!PyArg_ParseTuple(args, "y#y#K", &data, &data_len, &aad, &aad_len, &pn)) return NULL;
    if ((enc ? 0 : data_len < QPP_TAG_LEN) || data_len > QPP_PACKET_MAX || aad_len > QPP_MAX_HDR) {
        PyErr_SetString(g_crypto_error, "Invalid payload length");
        return NULL;
    }
    if (oneslot_ready(&self->s) < 0) return NULL;
    qpp_session *s = session();
    if (!s) return NULL;
    size_t in_len = (size_t)(aad_len + data_len);
    size_t out_len = in_len + (enc ? QPP_TAG_LEN : 0);
    unsigned char *buf = PyMem_Malloc(in_len + out_len + 1);
    if (!buf) return PyErr_NoMemory();
    memcpy(buf, aad, (size_t)aad_len);
    memcpy(buf + aad_len, data, (size_t)data_len);
    qpp_desc d;
    memset(&d, 0, sizeof d);
    d.len = (uint32_t)(enc ? data_len : aad_len + data_len);
    d.hdr_len = (uint16_t)aad_len;
    d.flags = QPP_F_NO_HP;
    d.pn = pn;
    qpp_result r;
    int rc = enc ? qpp_session_protect(s, self->s.kt, &d, 1, buf, in_len, buf + in_len, out_len, &r)
                 : qpp_session_unprotect(s, self->s.kt, &d, 1, buf, in_len, buf + in_len, out_len, &r);
    PyObject *ret = NULL;
    if (check_rc(rc) == 0) {
        if (r.status == QPP_S_OK)
            ret = PyBytes_FromStringAndSize((const char *)buf + in_len + aad_len,
                                            enc ? data_len + QPP_TAG_LEN : data_len - QPP_TAG_LEN);
        else if (r.status == QPP_S_DECRYPT)
            PyErr_SetString(g_crypto_error, "Payload decryption failed");
        else if (r.status == QPP_S_INTERNAL)
            PyErr_SetString(g_crypto_error, "Internal error: the packet was not processed");
        else
            PyErr_SetString(g_crypto_error, "Invalid payload length");
    }
    PyMem_Free(buf);
    return ret;
}

static PyObject *AEAD_encrypt(AEADObject *self, PyObject *args) { return aead_run(self, args, 1); }
static PyObject *AEAD_decrypt(AEADObject *self, PyObject *args) { return aead_run(self, args, 0); }

/* (suite, key, iv): lets the packet-level wrapper build fused key slots */
static PyObject *AEAD_material(AEADObject *self, PyObject *unused)
{
    int kl = suite_key_len(self->s.km.suite);
    return Py_BuildValue("iy#y#", (int)self->s.km.suite, self->s.km.key, (Py_ssize_t)kl,
                         self->s.km.iv, (Py_ssize_t)12);
}

static PyMethodDef AEAD_methods[] = {
    {"encrypt", (PyCFunction)AEAD_encrypt, METH_VARARGS, "encrypt(data, associated_data, packet_number) -> bytes"},
    {"decrypt", (PyCFunction)AEAD_decrypt, METH_VARARGS, "decrypt(data, associated_data, packet_number) -> bytes"},
    {"_material", (PyCFunction)AEAD_material, METH_NOARGS, "(suite, key, iv)"},
    {NULL},
};

static PyType_Slot AEAD_slots[] = {
    {Py_tp_doc, "AEAD payload protection on the GPU"},
    {Py_tp_methods, AEAD_methods},
    {Py_tp_init, AEAD_init},
    {Py_tp_new, PyType_GenericNew},
    {Py_tp_dealloc, AEAD_dealloc},
    {0, NULL},
};

static PyType_Spec AEAD_spec = {"aioquic_amd._crypto.AEAD", sizeof(AEADObject), 0,
                                Py_TPFLAGS_DEFAULT, AEAD_slots};

/* ---------------------------------------------------- HeaderProtection -- */

typedef struct {
    PyObject_HEAD
    OneSlot s;
} HPObject;

static int HP_init(HPObject *self, PyObject *args, PyObject *kwargs)
{
    const char *name;
    const unsigned char *key;
    Py_ssize_t name_len, key_len;
    if (!PyArg_ParseTuple(args, "y#y#", &name, &name_len, &key, &key_len)) return -1;
    int suite = hp_suite(name, name_len);
    if (suite < 0) {
        PyErr_Format(g_crypto_error, "Invalid cipher name: %s", name);
        return -1;
    }
    if (key_len != suite_key_len(suite)) {
        PyErr_SetString(g_crypto_error, "OpenSSL call failed");
        return -1;
    }
    oneslot_reset(&self->s, suite);
    memcpy(self->s.km.hp, key, (size_t)key_len);
    return oneslot_ready(&self->s);
}

static void HP_dealloc(HPObject *self)
{
    if (self->s.kt) qpp_keytab_destroy(self->s.kt);
    heap_dealloc((PyObject *)self);
}

static int hp_mask(HPObject *self, const unsigned char *sample, unsigned char mask[16])
{
    if (oneslot_ready(&self->s) < 0) return -1;
    qpp_session *s = session();
    if (!s) return -1;
    uint32_t slot = 0;
    return check_rc(qpp_session_hp_mask(s, self->s.kt, &slot, sample, 1, mask));
}

static unsigned char first_byte_bits(unsigned char b0) { return (b0 & 0x80) ? 0x0f : 0x1f; }

/* HeaderProtection.apply (_crypto.c:289-319) */
static PyObject *HP_apply(HPObject *self, PyObject *args)
{
    const unsigned char *hdr, *payload;
    Py_ssize_t hlen, plen;
    if (!PyArg_ParseTuple(args, "y#y#", &hdr, &hlen, &payload, &plen)) return NULL;
    if (hlen < 1) {
        PyErr_SetString(g_crypto_error, "Invalid payload length");
        return NULL;
    }
    int pn_len = (hdr[0] & 3) + 1;
    Py_ssize_t pn_off = hlen - pn_len;
    /* hlen + plen > 1500 overruns the reference's buffer (_crypto.c:305-306) */
    if (pn_off < 0 || plen < 20 - pn_len || hlen + plen > QPP_PACKET_MAX) {
        PyErr_SetString(g_crypto_error, "Invalid payload length");
        return NULL;
    }
    unsigned char mask[16];
    if (hp_mask(self, payload + 4 - pn_len, mask) < 0) return NULL;
    PyObject *out = PyBytes_FromStringAndSize(NULL, hlen + plen);
    if (!out) return NULL;
    unsigned char *o = (unsigned char *)PyBytes_AsString(out);
    memcpy(o, hdr, (size_t)hlen);
    memcpy(o + hlen, payload, (size_t)plen);
    o[0] ^= mask[0] & first_byte_bits(o[0]);
    for (int i = 0; i < pn_len; ++i) o[pn_off + i] ^= mask[1 + i];
    return out;
}

/* HeaderProtection.remove (_crypto.c:321-350): returns (header, truncated pn as C int) */
static PyObject *HP_remove(HPObject *self, PyObject *args)
{
    const unsigned char *pkt;
    Py_ssize_t len;
    unsigned int pn_off;
    if (!PyArg_ParseTuple(args, "y#I", &pkt, &len, &pn_off)) return NULL;
    if ((Py_ssize_t)pn_off + 20 > len) {
        PyErr_SetString(g_crypto_error, "Invalid payload length");
        return NULL;
    }
    unsigned char mask[16];
    if (hp_mask(self, pkt + pn_off + 4, mask) < 0) return NULL;
    unsigned char *buf = PyMem_Malloc((size_t)pn_off + 4);
    if (!buf) return PyErr_NoMemory();
    memcpy(buf, pkt, (size_t)pn_off + 4);
    buf[0] ^= mask[0] & first_byte_bits(buf[0]);
    int pn_len = (buf[0] & 3) + 1;
    uint32_t trunc = 0;
    for (int i = 0; i < pn_len; ++i) {
        buf[pn_off + i] ^= mask[1 + i];
        trunc = (trunc << 8) | buf[pn_off + i];
    }
    PyObject *ret = Py_BuildValue("y#i", buf, (Py_ssize_t)(pn_off + pn_len), (int)trunc);
    PyMem_Free(buf);
    return ret;
}

static PyObject *HP_material(HPObject *self, PyObject *unused)
{
    return Py_BuildValue("iy#", (int)self->s.km.suite, self->s.km.hp,
                         (Py_ssize_t)suite_key_len(self->s.km.suite));
}

static PyMethodDef HP_methods[] = {
    {"apply", (PyCFunction)HP_apply, METH_VARARGS, "apply(plain_header, protected_payload) -> bytes"},
    {"remove", (PyCFunction)HP_remove, METH_VARARGS, "remove(packet, encrypted_offset) -> (bytes, int)"},
    {"_material", (PyCFunction)HP_material, METH_NOARGS, "(suite, key)"},
    {NULL},
};

static PyType_Slot HP_slots[] = {
    {Py_tp_doc, "QUIC header protection masks on the GPU"},
    {Py_tp_methods, HP_methods},
    {Py_tp_init, HP_init},
    {Py_tp_new, PyType_GenericNew},
    {Py_tp_dealloc, HP_dealloc},
    {0, NULL},
};

static PyType_Spec HP_spec = {"aioquic_amd._crypto.HeaderProtection", sizeof(HPObject), 0,
                              Py_TPFLAGS_DEFAULT, HP_slots};

/* ------------------------------------------------------------ KeyTable -- */

typedef struct {
    PyObject_HEAD
    qpp_keytab *kt;
} KeyTableObject;

static int KT_init(KeyTableObject *self, PyObject *args, PyObject *kwargs)
{
    unsigned int cap;
    if (!PyArg_ParseTuple(args, "I", &cap)) return -1;
    if (self->kt) {
        qpp_keytab_destroy(self->kt);
        self->kt = NULL;
    }
    int rc = qpp_keytab_create(cap, &self->kt);
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "invalid key-table capacity");
        return -1;
    }
    return check_rc(rc);
}

static void KT_dealloc(KeyTableObject *self)
{
    if (self->kt) qpp_keytab_destroy(self->kt);
    heap_dealloc((PyObject *)self);
}

/* set(materials: bytes-like of n packed qpp_key_material records, stream=0) */
static PyObject *KT_set(KeyTableObject *self, PyObject *args)
{
    const char *b;
    Py_ssize_t len;
    unsigned long long stream = 0;
    if (!PyArg_ParseTuple(args, "y#|K", &b, &len, &stream)) return NULL;
    if (len % (Py_ssize_t)sizeof(qpp_key_material)) {
        PyErr_SetString(PyExc_ValueError, "materials must be a whole number of 84-byte records");
        return NULL;
    }
    uint32_t n = (uint32_t)(len / (Py_ssize_t)sizeof(qpp_key_material));
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_keytab_set(self->kt, (const qpp_key_material *)b, n, as_ptr(stream));
    Py_END_ALLOW_THREADS
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "bad key material (slot out of range or unknown suite)");
        return NULL;
    }
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

/* KeyTable.derive(secrets) -> key material: batched CryptoContext.setup
 * (qpp_keytab_derive); secrets = whole qpp_secret records. */
static PyObject *KT_derive(KeyTableObject *self, PyObject *args)
{
    const char *b;
    Py_ssize_t len;
    unsigned long long stream = 0;
    if (!PyArg_ParseTuple(args, "y#|K", &b, &len, &stream)) return NULL;
    if (len % (Py_ssize_t)sizeof(qpp_secret)) {
        PyErr_SetString(PyExc_ValueError, "secrets must be a whole number of 80-byte records");
        return NULL;
    }
    uint32_t n = (uint32_t)(len / (Py_ssize_t)sizeof(qpp_secret));
    PyObject *km = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * (Py_ssize_t)sizeof(qpp_key_material));
    if (!km) return NULL;
    qpp_key_material *out = (qpp_key_material *)PyBytes_AsString(km);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_keytab_derive(self->kt, (const qpp_secret *)b, n, out, as_ptr(stream));
    Py_END_ALLOW_THREADS
    if (rc == QPP_E_ARG) {
        Py_DECREF(km);
        PyErr_SetString(PyExc_ValueError, "bad secret (slot out of range, unknown suite or length)");
        return NULL;
    }
    if (check_rc(rc) < 0) {
        Py_DECREF(km);
        return NULL;
    }
    return km;
}

static PyObject *KT_clear(KeyTableObject *self, PyObject *args)
{
    const char *b;
    Py_ssize_t len;
    if (!PyArg_ParseTuple(args, "y#", &b, &len)) return NULL;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_keytab_clear(self->kt, (const uint32_t *)b, (uint32_t)(len / 4), NULL);
    Py_END_ALLOW_THREADS
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

static PyObject *KT_capacity(KeyTableObject *self, void *unused)
{
    return PyLong_FromUnsignedLong(qpp_keytab_capacity(self->kt));
}

static PyMethodDef KT_methods[] = {
    {"set", (PyCFunction)KT_set, METH_VARARGS, "set(materials, stream=0)"},
    {"clear", (PyCFunction)KT_clear, METH_VARARGS, "clear(slots_u32)"},
    {"derive", (PyCFunction)KT_derive, METH_VARARGS, "derive(secrets, stream=0) -> key material"},
    {NULL},
};

static PyGetSetDef KT_getset[] = {
    {"capacity", (getter)KT_capacity, NULL, "number of key slots", NULL},
    {NULL},
};

static PyType_Slot KT_slots[] = {
    {Py_tp_doc, "device-resident expanded key slots"},
    {Py_tp_methods, KT_methods},
    {Py_tp_getset, KT_getset},
    {Py_tp_init, KT_init},
    {Py_tp_new, PyType_GenericNew},
    {Py_tp_dealloc, KT_dealloc},
    {0, NULL},
};

static PyType_Spec KT_spec = {"aioquic_amd._crypto.KeyTable", sizeof(KeyTableObject), 0,
                              Py_TPFLAGS_DEFAULT, KT_slots};

static qpp_keytab *as_table(PyObject *o)
{
    if (!PyObject_TypeCheck(o, (PyTypeObject *)g_kt_type)) {
        PyErr_SetString(PyExc_TypeError, "expected a KeyTable");
        return NULL;
    }
    return ((KeyTableObject *)o)->kt;
}

/* ---------------------------------------------------------------- Plan -- */

typedef struct {
    PyObject_HEAD
    qpp_plan *plan;
} PlanObject;

static int Plan_init(PlanObject *self, PyObject *args, PyObject *kwargs)
{
    unsigned int cap;
    if (!PyArg_ParseTuple(args, "I", &cap)) return -1;
    if (self->plan) {
        qpp_plan_destroy(self->plan);
        self->plan = NULL;
    }
    int rc = qpp_plan_create(cap, &self->plan);
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "invalid plan capacity");
        return -1;
    }
    return check_rc(rc);
}

static void Plan_dealloc(PlanObject *self)
{
    if (self->plan) qpp_plan_destroy(self->plan);
    heap_dealloc((PyObject *)self);
}

static PyType_Slot Plan_slots[] = {
    {Py_tp_doc, "device scratch of the (suite, key slot) bucketing step"},
    {Py_tp_init, Plan_init},
    {Py_tp_new, PyType_GenericNew},
    {Py_tp_dealloc, Plan_dealloc},
    {0, NULL},
};

static PyType_Spec Plan_spec = {"aioquic_amd._crypto.Plan", sizeof(PlanObject), 0,
                                Py_TPFLAGS_DEFAULT, Plan_slots};

/* NULL for None, else the plan (NULL with an exception set for a wrong type) */
static int as_plan(PyObject *o, qpp_plan **out)
{
    *out = NULL;
    if (!o || o == Py_None) return 0;
    if (!PyObject_TypeCheck(o, (PyTypeObject *)g_plan_type)) {
        PyErr_SetString(PyExc_TypeError, "expected a Plan or None");
        return -1;
    }
    *out = ((PlanObject *)o)->plan;
    return 0;
}

/* --------------------------------------------------------- MultiSession -- */

/* MultiSession(devices, key_capacity): one host batch over several GPUs
 * (qpp_multi, quic_pp.h).  .set_keys(materials), .protect(desc, data,
 * out_len) / .unprotect(...) -> (out, results) like protect_host; .devices. */
typedef struct {
    PyObject_HEAD
    qpp_multi *m;
} MultiObject;

static int Multi_init(MultiObject *self, PyObject *args, PyObject *kwargs)
{
    PyObject *devs;
    unsigned int cap;
    if (!PyArg_ParseTuple(args, "OI", &devs, &cap)) return -1;
    const Py_ssize_t nd = PySequence_Size(devs);
    int ids[16];
    if (nd < 0) return -1;
    if (nd < 1 || nd > 16) {
        PyErr_SetString(PyExc_ValueError, "1 to 16 devices");
        return -1;
    }
    for (Py_ssize_t k = 0; k < nd; ++k) {
        PyObject *it = PySequence_GetItem(devs, k);
        if (!it) return -1;
        ids[k] = (int)PyLong_AsLong(it);
        Py_DECREF(it);
        if (ids[k] == -1 && PyErr_Occurred()) return -1;
    }
    if (self->m) {
        qpp_multi_destroy(self->m);
        self->m = NULL;
    }
    int rc = qpp_multi_create(ids, (int)nd, cap, &self->m);
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "bad device list or key capacity");
        return -1;
    }
    return check_rc(rc);
}

static void Multi_dealloc(MultiObject *self)
{
    if (self->m) qpp_multi_destroy(self->m);
    heap_dealloc((PyObject *)self);
}

static PyObject *Multi_set_keys(MultiObject *self, PyObject *args)
{
    const char *b;
    Py_ssize_t len;
    if (!PyArg_ParseTuple(args, "y#", &b, &len)) return NULL;
    if (len % (Py_ssize_t)sizeof(qpp_key_material)) {
        PyErr_SetString(PyExc_ValueError, "materials must be a whole number of 84-byte records");
        return NULL;
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_multi_set_keys(self->m, (const qpp_key_material *)b, (uint32_t)(len / (Py_ssize_t)sizeof(qpp_key_material)));
    Py_END_ALLOW_THREADS
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "bad key material (slot out of range or unknown suite)");
        return NULL;
    }
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

static PyObject *multi_run_py(MultiObject *self, PyObject *args, int enc)
{
    const char *desc, *data;
    Py_ssize_t desc_len, data_len, out_len;
    if (!PyArg_ParseTuple(args, "y#y#n", &desc, &desc_len, &data, &data_len, &out_len)) return NULL;
    if (desc_len % (Py_ssize_t)sizeof(qpp_desc) || out_len < 0) {
        PyErr_SetString(PyExc_ValueError, "bad descriptor buffer or output length");
        return NULL;
    }
    const uint32_t n = (uint32_t)(desc_len / (Py_ssize_t)sizeof(qpp_desc));
    PyObject *out = PyBytes_FromStringAndSize(NULL, out_len);
    PyObject *res = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * (Py_ssize_t)sizeof(qpp_result));
    PyObject *ret = NULL;
    if (out && res) {
        int rc;
        char *o = PyBytes_AsString(out), *r = PyBytes_AsString(res);
        Py_BEGIN_ALLOW_THREADS
        rc = enc ? qpp_multi_protect(self->m, (const qpp_desc *)desc, n, (const uint8_t *)data, (size_t)data_len,
                                     (uint8_t *)o, (size_t)out_len, (qpp_result *)r)
                 : qpp_multi_unprotect(self->m, (const qpp_desc *)desc, n, (const uint8_t *)data, (size_t)data_len,
                                       (uint8_t *)o, (size_t)out_len, (qpp_result *)r);
        Py_END_ALLOW_THREADS
        if (check_rc(rc) == 0) ret = PyTuple_Pack(2, out, res);
    }
    Py_XDECREF(out);
    Py_XDECREF(res);
    return ret;
}

static PyObject *Multi_protect(MultiObject *self, PyObject *args) { return multi_run_py(self, args, 1); }
static PyObject *Multi_unprotect(MultiObject *self, PyObject *args) { return multi_run_py(self, args, 0); }

/* protect_into / unprotect_into(desc_ptr, n, in_ptr, in_len, out_ptr, out_len,
 * res_ptr): host memory by address (caller-owned, reused across batches). */
static PyObject *multi_into_py(MultiObject *self, PyObject *args, int enc)
{
    unsigned long long dp, ip, op, rp, in_len, out_len;
    unsigned int n;
    if (!PyArg_ParseTuple(args, "KIKKKKK", &dp, &n, &ip, &in_len, &op, &out_len, &rp)) return NULL;
    if (n && (!dp || !rp || (in_len && !ip) || (out_len && !op))) {
        PyErr_SetString(PyExc_ValueError, "null buffer");
        return NULL;
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = enc ? qpp_multi_protect(self->m, (const qpp_desc *)as_ptr(dp), n, (const uint8_t *)as_ptr(ip),
                                 (size_t)in_len, (uint8_t *)as_ptr(op), (size_t)out_len, (qpp_result *)as_ptr(rp))
             : qpp_multi_unprotect(self->m, (const qpp_desc *)as_ptr(dp), n, (const uint8_t *)as_ptr(ip),
                                   (size_t)in_len, (uint8_t *)as_ptr(op), (size_t)out_len, (qpp_result *)as_ptr(rp));
    Py_END_ALLOW_THREADS
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

static PyObject *Multi_protect_into(MultiObject *self, PyObject *args) { return multi_into_py(self, args, 1); }
static PyObject *Multi_unprotect_into(MultiObject *self, PyObject *args) { return multi_into_py(self, args, 0); }

/* trace(enable=-1) -> [dict per device]: the phases of each device session's
 * last traced pipelined call (qpp_multi_trace); enable 1 / 0 turns tracing
 * on / off for the following calls. */
static PyObject *Multi_trace(MultiObject *self, PyObject *args)
{
    int enable = -1;
    if (!PyArg_ParseTuple(args, "|i", &enable)) return NULL;
    qpp_trace t[16];
    const int k = qpp_multi_trace(self->m, enable, t, 16);
    if (k < 0) {
        check_rc(k);
        return NULL;
    }
    PyObject *lst = PyList_New(0);
    for (int i = 0; lst && i < k; ++i) {
        PyObject *d = Py_BuildValue(
            "{s:I,s:I,s:d,s:d,s:d,s:d,s:d,s:d,s:d,s:d,s:d,s:d,s:d}", "pipelined", t[i].pipelined, "chunks",
            t[i].chunks, "total_ms", t[i].total_ms, "submit_ms", t[i].submit_ms, "copy_in_ms", t[i].copy_in_ms,
            "copy_out_ms", t[i].copy_out_ms, "wait_ms", t[i].wait_ms, "h2d_ms", t[i].h2d_ms, "kernel_ms",
            t[i].kernel_ms, "d2h_ms", t[i].d2h_ms, "gpu_span_ms", t[i].gpu_span_ms, "in_bytes", t[i].in_bytes,
            "out_bytes", t[i].out_bytes);
        if (!d || PyList_Append(lst, d) < 0) {
            Py_XDECREF(d);
            Py_DECREF(lst);
            return NULL;
        }
        Py_DECREF(d);
    }
    return lst;
}

static PyObject *Multi_devices(MultiObject *self, void *unused)
{
    return PyLong_FromLong(qpp_multi_devices(self->m));
}

static PyMethodDef Multi_methods[] = {
    {"set_keys", (PyCFunction)Multi_set_keys, METH_VARARGS, "set_keys(materials) on every device"},
    {"protect", (PyCFunction)Multi_protect, METH_VARARGS, "protect(desc, data, out_len) -> (out, results)"},
    {"unprotect", (PyCFunction)Multi_unprotect, METH_VARARGS, "unprotect(desc, data, out_len) -> (out, results)"},
    {"protect_into", (PyCFunction)Multi_protect_into, METH_VARARGS,
     "protect_into(desc_ptr, n, in_ptr, in_len, out_ptr, out_len, res_ptr)"},
    {"unprotect_into", (PyCFunction)Multi_unprotect_into, METH_VARARGS,
     "unprotect_into(desc_ptr, n, in_ptr, in_len, out_ptr, out_len, res_ptr)"},
    {"trace", (PyCFunction)Multi_trace, METH_VARARGS,
     "trace(enable=-1) -> per device, the last traced call's host / PCIe / kernel phases"},
    {NULL},
};

static PyGetSetDef Multi_getset[] = {
    {"devices", (getter)Multi_devices, NULL, "number of device sessions", NULL},
    {NULL},
};

static PyType_Slot Multi_slots[] = {
    {Py_tp_doc, "one host batch over several GPUs (qpp_multi)"},
    {Py_tp_methods, Multi_methods},
    {Py_tp_getset, Multi_getset},
    {Py_tp_init, Multi_init},
    {Py_tp_new, PyType_GenericNew},
    {Py_tp_dealloc, Multi_dealloc},
    {0, NULL},
};

static PyType_Spec Multi_spec = {"aioquic_amd._crypto.MultiSession", sizeof(MultiObject), 0,
                                 Py_TPFLAGS_DEFAULT, Multi_slots};

/* -------------------------------------------------------- batch calls -- */

/* protect / unprotect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream[, plan]) */
static PyObject *batch_dev(PyObject *args, int enc)
{
    PyObject *t, *po = NULL;
    unsigned long long dp, ip, op, rp, sp;
    unsigned int n;
    if (!PyArg_ParseTuple(args, "OKIKKKK|O", &t, &dp, &n, &ip, &op, &rp, &sp, &po)) return NULL;
    qpp_keytab *kt = as_table(t);
    qpp_plan *plan;
    if (!kt || as_plan(po, &plan) < 0) return NULL;
    int rc = plan ? (enc ? qpp_protect_planned : qpp_unprotect_planned)(
                        kt, plan, as_ptr(dp), n, as_ptr(ip), as_ptr(op), as_ptr(rp), as_ptr(sp))
                  : (enc ? qpp_protect : qpp_unprotect)(kt, as_ptr(dp), n, as_ptr(ip), as_ptr(op),
                                                        as_ptr(rp), as_ptr(sp));
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "bad batch arguments (n beyond the plan's capacity?)");
        return NULL;
    }
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

static PyObject *py_protect(PyObject *m, PyObject *args) { return batch_dev(args, 1); }
static PyObject *py_unprotect(PyObject *m, PyObject *args) { return batch_dev(args, 0); }

/* plan_build(plan, table, desc_ptr, n, stream) */
static PyObject *py_plan_build(PyObject *m, PyObject *args)
{
    PyObject *po, *t;
    unsigned long long dp, sp;
    unsigned int n;
    if (!PyArg_ParseTuple(args, "OOKIK", &po, &t, &dp, &n, &sp)) return NULL;
    qpp_keytab *kt = as_table(t);
    qpp_plan *plan;
    if (!kt || as_plan(po, &plan) < 0) return NULL;
    if (!plan) {
        PyErr_SetString(PyExc_TypeError, "expected a Plan");
        return NULL;
    }
    int rc = qpp_plan_build(plan, kt, as_ptr(dp), n, as_ptr(sp));
    if (rc == QPP_E_ARG) {
        PyErr_SetString(PyExc_ValueError, "batch larger than the plan's capacity");
        return NULL;
    }
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

static int host_call(int enc, qpp_keytab *kt, const void *desc, uint32_t n, const void *in,
                     size_t in_len, void *out, size_t out_len, void *res)
{
    qpp_session *s = session();
    if (!s) return -1;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = enc ? qpp_session_protect(s, kt, desc, n, in, in_len, out, out_len, res)
             : qpp_session_unprotect(s, kt, desc, n, in, in_len, out, out_len, res);
    Py_END_ALLOW_THREADS
    return check_rc(rc);
}

/* protect_host / unprotect_host(table, desc, data, out_len) -> (out, results) */
static PyObject *batch_host(PyObject *args, int enc)
{
    PyObject *t;
    const char *desc, *data;
    Py_ssize_t desc_len, data_len, out_len;
    if (!PyArg_ParseTuple(args, "Oy#y#n", &t, &desc, &desc_len, &data, &data_len, &out_len))
        return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    if (desc_len % (Py_ssize_t)sizeof(qpp_desc) || out_len < 0) {
        PyErr_SetString(PyExc_ValueError, "bad descriptor buffer or output length");
        return NULL;
    }
    uint32_t n = (uint32_t)(desc_len / (Py_ssize_t)sizeof(qpp_desc));
    PyObject *out = PyBytes_FromStringAndSize(NULL, out_len);
    PyObject *res = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * (Py_ssize_t)sizeof(qpp_result));
    PyObject *ret = NULL;
    if (out && res) {
        char *o = PyBytes_AsString(out);
        /* the session writes every byte of out (zeros where no packet lands)
           for n > 0, so only an empty batch needs the zero fill here */
        if (n == 0) memset(o, 0, (size_t)out_len);
        if (host_call(enc, kt, desc, n, data, (size_t)data_len, o, (size_t)out_len,
                      PyBytes_AsString(res)) == 0)
            ret = PyTuple_Pack(2, out, res);
    }
    Py_XDECREF(out);
    Py_XDECREF(res);
    return ret;
}

static PyObject *py_protect_host(PyObject *m, PyObject *args) { return batch_host(args, 1); }
static PyObject *py_unprotect_host(PyObject *m, PyObject *args) { return batch_host(args, 0); }

/* protect_into / unprotect_into(table, desc_ptr, n, in_ptr, in_len, out_ptr,
   out_len, res_ptr): host memory given by address (e.g. numpy arrays reused
   across batches), so a large batch neither allocates nor first-touches a
   fresh bytes object per call.  The caller keeps the memory alive. */
static PyObject *batch_into(PyObject *args, int enc)
{
    PyObject *t;
    unsigned long long dp, ip, op, rp, in_len, out_len;
    unsigned int n;
    if (!PyArg_ParseTuple(args, "OKIKKKKK", &t, &dp, &n, &ip, &in_len, &op, &out_len, &rp))
        return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    if (n == 0) {
        if (out_len) memset(as_ptr(op), 0, (size_t)out_len);
        Py_RETURN_NONE;
    }
    if (!dp || !rp || (in_len && !ip) || (out_len && !op)) {
        PyErr_SetString(PyExc_ValueError, "null buffer");
        return NULL;
    }
    if (host_call(enc, kt, as_ptr(dp), n, as_ptr(ip), (size_t)in_len, as_ptr(op), (size_t)out_len,
                  as_ptr(rp)) < 0)
        return NULL;
    Py_RETURN_NONE;
}

static PyObject *py_protect_into(PyObject *m, PyObject *args) { return batch_into(args, 1); }
static PyObject *py_unprotect_into(PyObject *m, PyObject *args) { return batch_into(args, 0); }

/* protect_list(table, slots_u32, pns_u64, headers, payloads) -> (wires, results)
 * unprotect_list(table, slots_u32, expected_u64, packets, pn_offs_u32)
 *     -> (list of (plain_header, payload) or None, results)
 * The batched callers' form: the packets are copied straight from the bytes
 * objects of the lists into the session's pinned staging buffer, and the
 * outputs are cut straight from its pinned output buffer, one bytes object
 * each; no intermediate joins or slices in Python. */
static PyObject *batch_list(PyObject *args, int enc)
{
    PyObject *t, *items;
    const char *slots, *nums, *extra = NULL;
    Py_ssize_t slots_len, nums_len, extra_len = 0;
    PyObject *payloads = NULL;
    if (enc) {
        if (!PyArg_ParseTuple(args, "Oy#y#O!O!", &t, &slots, &slots_len, &nums, &nums_len, &PyList_Type,
                              &items, &PyList_Type, &payloads))
            return NULL;
    } else if (!PyArg_ParseTuple(args, "Oy#y#O!y#", &t, &slots, &slots_len, &nums, &nums_len, &PyList_Type,
                                 &items, &extra, &extra_len)) {
        return NULL;
    }
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    const Py_ssize_t n = PyList_Size(items);
    if (slots_len != 4 * n || nums_len != 8 * n || (enc ? PyList_Size(payloads) != n : extra_len != 4 * n)) {
        PyErr_SetString(PyExc_ValueError, "per-packet arrays do not match the packet list");
        return NULL;
    }
    if (n > 0x7fffffff) {
        PyErr_SetString(PyExc_ValueError, "batch too large");
        return NULL;
    }
    /* first pass: sizes (and the type check of every item) */
    size_t total = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
        char *b;
        Py_ssize_t l1, l2 = 0;
        if (PyBytes_AsStringAndSize(PyList_GetItem(items, i), &b, &l1) < 0) return NULL;
        if (enc && PyBytes_AsStringAndSize(PyList_GetItem(payloads, i), &b, &l2) < 0) return NULL;
        /* protect: up to 15 bytes of room to start each payload on a
           16-byte boundary (Payload alignment) */
        total += (size_t)l1 + (size_t)l2 + (enc ? QPP_TAG_LEN + 15 : 0);
    }
    qpp_session *s = session();
    if (!s) return NULL;
    PyObject *res = PyBytes_FromStringAndSize(NULL, n * (Py_ssize_t)sizeof(qpp_result));
    qpp_desc *desc = (qpp_desc *)calloc(n ? (size_t)n : 1, sizeof(qpp_desc));
    uint8_t *hin = NULL, *hout = NULL;
    PyObject *ret = NULL, *outs = NULL;
    if (!res || !desc) {
        PyErr_NoMemory();
        goto done;
    }
    if (n == 0) {
        outs = PyList_New(0);
        goto pack;
    }
    if (check_rc(qpp_session_stage(s, total ? total : 1, (uint32_t)n, &hin, &hout)) < 0) goto done;
    {
        const uint32_t *sl = (const uint32_t *)slots;
        size_t off = 0;
        for (Py_ssize_t i = 0; i < n; ++i) {
            char *b1, *b2 = NULL;
            Py_ssize_t l1, l2 = 0;
            (void)PyBytes_AsStringAndSize(PyList_GetItem(items, i), &b1, &l1);
            if (enc) (void)PyBytes_AsStringAndSize(PyList_GetItem(payloads, i), &b2, &l2);
            qpp_desc *d = &desc[i];
            if (enc) off = ((off + (size_t)l1 + 15) & ~(size_t)15) - (size_t)l1;
            d->in_off = d->out_off = off;
            uint64_t num;
            memcpy(&num, nums + 8 * i, 8);
            d->pn = num;
            d->slot = sl[i];
            memcpy(hin + off, b1, (size_t)l1);
            if (enc) {
                /* a header the 16-bit field cannot carry is rejected below */
                d->hdr_len = l1 > 0xffff ? 0xffff : (uint16_t)l1;
                d->len = (uint32_t)l2;
                memcpy(hin + off + l1, b2, (size_t)l2);
                off += (size_t)l1 + (size_t)l2 + QPP_TAG_LEN;
            } else {
                uint32_t po;
                memcpy(&po, extra + 4 * i, 4);
                d->hdr_len = po > 0xffff ? 0xffff : (uint16_t)po;
                d->len = (uint32_t)l1;
                off += (size_t)l1;
            }
        }
    }
    if (host_call(enc, kt, desc, (uint32_t)n, hin, total, hout, total, PyBytes_AsString(res)) < 0) goto done;
    outs = PyList_New(n);
    if (!outs) goto done;
    {
        const qpp_result *r = (const qpp_result *)PyBytes_AsString(res);
        for (Py_ssize_t i = 0; i < n; ++i) {
            const uint8_t *o = hout + desc[i].out_off;
            PyObject *item;
            if (enc) {
                item = PyBytes_FromStringAndSize((const char *)o, (Py_ssize_t)desc[i].hdr_len + desc[i].len +
                                                                      QPP_TAG_LEN);
            } else if (r[i].status == QPP_S_OK) {
                PyObject *h = PyBytes_FromStringAndSize((const char *)o, r[i].hdr_len);
                PyObject *p = PyBytes_FromStringAndSize((const char *)o + r[i].hdr_len,
                                                        (Py_ssize_t)r[i].out_len - r[i].hdr_len);
                item = (h && p) ? PyTuple_Pack(2, h, p) : NULL;
                Py_XDECREF(h);
                Py_XDECREF(p);
                if (item) PyObject_GC_UnTrack(item); /* two bytes objects: never in a cycle */
            } else {
                Py_INCREF(Py_None);
                item = Py_None;
            }
            if (!item) {
                Py_CLEAR(outs);
                goto done;
            }
            PyList_SetItem(outs, i, item); /* steals */
        }
    }
pack:
    if (outs) ret = PyTuple_Pack(2, outs, res);
done:
    Py_XDECREF(outs);
    Py_XDECREF(res);
    free(desc);
    return ret;
}

static PyObject *py_protect_list(PyObject *m, PyObject *args) { return batch_list(args, 1); }
static PyObject *py_unprotect_list(PyObject *m, PyObject *args) { return batch_list(args, 0); }

/* A per-packet array argument ("y#": any read-only bytes-like object)
 * must hold exactly n items of `size` bytes. */
static int check_len(Py_ssize_t len, Py_ssize_t n, Py_ssize_t size, const char *what)
{
    if (len == n * size) return 0;
    PyErr_Format(PyExc_ValueError, "%s: %zd bytes for %zd items of %zd", what, len, n, size);
    return -1;
}

/* protect_datagrams(table, plains, dg_u32, off_u32, hsize_u32, size_u32, pn_u64, slot_u32)
 *     -> (wire datagrams, results)
 * The deferred-encryption builder's flush (QuicPacketBuilder._end_packet,
 * packet_builder.py:341-350, for every packet of every datagram at once):
 * the plaintext datagrams go back to back into the session's pinned staging;
 * packet k of datagram dg[k] starts at off[k] with hsize[k] header bytes and
 * size[k] header + payload bytes (its tag's room follows).  Each wire
 * datagram comes back as one bytes object cut from the pinned output, which
 * the session writes in full (zeros outside packets: the builder's datagram
 * padding is zeros too). */
static PyObject *py_protect_datagrams(PyObject *m, PyObject *args)
{
    PyObject *t, *plains;
    const char *a_dg, *a_off, *a_hs, *a_sz, *a_pn, *a_sl;
    Py_ssize_t l_dg, l_off, l_hs, l_sz, l_pn, l_sl;
    if (!PyArg_ParseTuple(args, "OO!y#y#y#y#y#y#", &t, &PyList_Type, &plains, &a_dg, &l_dg, &a_off, &l_off, &a_hs,
                          &l_hs, &a_sz, &l_sz, &a_pn, &l_pn, &a_sl, &l_sl))
        return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    const Py_ssize_t n = l_dg / 4;
    if (check_len(l_dg, n, 4, "dg") < 0 || check_len(l_off, n, 4, "off") < 0 || check_len(l_hs, n, 4, "hsize") < 0 ||
        check_len(l_sz, n, 4, "size") < 0 || check_len(l_pn, n, 8, "pn") < 0 || check_len(l_sl, n, 4, "slot") < 0)
        return NULL;
    /* a snapshot holding a reference to every datagram: the copies below run
       without the GIL, while another thread may change the caller's list */
    plains = PySequence_Tuple(plains);
    if (!plains) return NULL;
    const Py_ssize_t nd = PyTuple_Size(plains);
    PyObject *ret = NULL, *wires = NULL, *res = NULL;
    size_t *base = NULL;
    qpp_desc *desc = NULL;
    base = (size_t *)malloc(((size_t)nd + 1) * sizeof(size_t));
    desc = (qpp_desc *)calloc(n ? (size_t)n : 1, sizeof(qpp_desc));
    res = PyBytes_FromStringAndSize(NULL, n * (Py_ssize_t)sizeof(qpp_result));
    if (!base || !desc || !res) {
        PyErr_NoMemory();
        goto done;
    }
    base[0] = 0;
    for (Py_ssize_t d = 0; d < nd; ++d) {
        PyObject *o = PyTuple_GetItem(plains, d);
        if (!PyBytes_Check(o)) {
            PyErr_SetString(PyExc_TypeError, "datagrams must be bytes");
            goto done;
        }
        base[d + 1] = base[d] + (size_t)PyBytes_Size(o);
    }
    {
        const uint32_t *dg = (const uint32_t *)a_dg, *off = (const uint32_t *)a_off, *hs = (const uint32_t *)a_hs,
                       *sz = (const uint32_t *)a_sz, *sl = (const uint32_t *)a_sl;
        const uint64_t *pn = (const uint64_t *)a_pn;
        for (Py_ssize_t k = 0; k < n; ++k) {
            if (dg[k] >= (uint32_t)nd || hs[k] > sz[k] ||
                (size_t)off[k] + sz[k] + QPP_TAG_LEN > base[dg[k] + 1] - base[dg[k]]) {
                PyErr_SetString(PyExc_ValueError, "packet outside its datagram");
                goto done;
            }
            qpp_desc *x = &desc[k];
            x->in_off = x->out_off = base[dg[k]] + off[k];
            x->hdr_len = hs[k] > 0xffff ? 0xffff : (uint16_t)hs[k];
            x->len = sz[k] - hs[k];
            x->pn = pn[k];
            x->slot = sl[k];
        }
    }
    {
        const size_t total = base[nd];
        qpp_session *s = session();
        uint8_t *hin, *hout;
        if (!s || check_rc(qpp_session_stage(s, total ? total : 1, (uint32_t)(n ? n : 1), &hin, &hout)) < 0)
            goto done;
        /* the copy jobs: datagram d between its bytes object and staging */
        uint8_t **cd = (uint8_t **)malloc(((size_t)nd + 1) * sizeof(uint8_t *));
        const uint8_t **cs = (const uint8_t **)malloc(((size_t)nd + 1) * sizeof(uint8_t *));
        size_t *cl = (size_t *)malloc(((size_t)nd + 1) * sizeof(size_t));
        if (!cd || !cs || !cl) {
            free(cd), free(cs), free(cl);
            PyErr_NoMemory();
            goto done;
        }
        for (Py_ssize_t d = 0; d < nd; ++d) {
            cd[d] = hin + base[d];
            cs[d] = (const uint8_t *)PyBytes_AsString(PyTuple_GetItem(plains, d));
            cl[d] = base[d + 1] - base[d];
        }
        Py_BEGIN_ALLOW_THREADS  /* the snapshot holds every datagram */
        par_copy(cd, cs, cl, (size_t)nd, total);
        Py_END_ALLOW_THREADS
        const uint8_t *src = hin;  /* no packet: the datagrams as they are */
        int ok = 1;
        if (n) {
            ok = host_call(1, kt, desc, (uint32_t)n, hin, total, hout, total, PyBytes_AsString(res)) == 0;
            src = hout;
        }
        if (ok) wires = PyList_New(nd);
        for (Py_ssize_t d = 0; wires && d < nd; ++d) {
            /* allocated here, filled below without the GIL (not yet shared) */
            PyObject *o = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)cl[d]);
            if (!o) {
                Py_CLEAR(wires);
                break;
            }
            PyList_SetItem(wires, d, o);
            cd[d] = (uint8_t *)PyBytes_AsString(o);
            cs[d] = src + base[d];
        }
        if (wires) {
            Py_BEGIN_ALLOW_THREADS
            par_copy(cd, cs, cl, (size_t)nd, total);
            Py_END_ALLOW_THREADS
            ret = PyTuple_Pack(2, wires, res);
        }
        free(cd), free(cs), free(cl);
    }
done:
    Py_XDECREF(wires);
    Py_XDECREF(res);
    Py_DECREF(plains);
    free(base);
    free(desc);
    return ret;
}

/* Host-side outcomes of the receive walks (never produced by a kernel):
 * a packet that authenticated with a reserved bit set (connection.py:949-960),
 * a packet of a connection the walk has closed (:756-757). */
#define WALK_S_RESERVED 0x101
#define WALK_S_CLOSED 0x102
#define WALK_NO_CONN 0xffffffffu
/* receive_short's slot_of: closed on entry / no receive key (no launch) */
#define RS_CLOSED 0xfffffffeu

/* decode_packet_number (quic/packet.py:118-132) of the truncated number as
 * HeaderProtection.remove hands it over: a signed C int (_crypto.c:349), so a
 * 4-byte value >= 2^31 enters negative, exactly as the Python walk sees it.
 * Returns -1 where Python would produce a negative number. */
static int64_t decode_pn_signed(uint64_t pn, int pn_len, uint64_t expected)
{
    const int bits = 8 * pn_len;
    int64_t trunc = (int64_t)(pn & ((1ull << bits) - 1));
    if (pn_len == 4 && trunc >= ((int64_t)1 << 31)) trunc -= (int64_t)1 << 32;
    const int64_t window = (int64_t)1 << bits, half = window / 2, exp = (int64_t)expected;
    const int64_t cand = (exp & ~(window - 1)) | trunc;
    int64_t r;
    if (cand <= exp - half && cand < ((int64_t)1 << 62) - window) r = cand + window;
    else if (cand > exp + half && cand >= window) r = cand - window;
    else r = cand;
    return r < 0 ? -1 : r;
}

/* unprotect_walk(table, slots_u32, exp_u64, packets, offs_u32, pair_u32,
 *                space_u32, track_u8, space_exp_u64, n_pairs, conn_u32,
 *                rsv_u8, closed_u8)
 *     -> (outcomes, results, deferred, space_exp_u64 after the walk,
 *         closed_u8 after the walk)
 * One ReceiveBatch round in C: the launch (as unprotect_list, each packet
 * decoded against exp[i], its space's expected number when the round began)
 * and the in-order walk of CryptoPair.decrypt_packet semantics
 * (quic/crypto.py:184-192, connection.py:905-947,984-985) for every packet
 * whose outcome does not depend on a state change this round makes:
 *   outcomes[i] = (plain_header, payload, packet_number) on success, None on
 *   failure (results[i].status says which), or None for a deferred packet;
 *   the returned copy of space_exp advances as connection.py:984-985 does
 *   (for track[i]).
 * A packet is deferred -- and with it every later packet of its pair and of
 * its space -- when its key phase flipped (a key roll follows), or when its
 * truncated number decodes differently under the space's expected number by
 * now than under exp[i].  The caller's general walk (batch_io.ReceiveBatch)
 * then continues with the deferred packets, in order, from the state left
 * here.
 * Connections (conn_u32[i]: the packet's connection, WALK_NO_CONN for none;
 * rsv_u8[i]: its reserved-bit mask, 0 for no check; closed_u8: each
 * connection's closed flag, returned updated): a packet that authenticates
 * with a reserved bit set closes its connection (connection.py:949-960) --
 * status WALK_S_RESERVED, no expected-number update -- and every later packet
 * of a closed connection gets WALK_S_CLOSED (:756-757).  A deferred packet
 * blocks its connection too: whether it closes it is not known yet. */
static PyObject *py_unprotect_walk(PyObject *m, PyObject *args)
{
    PyObject *t, *packets;
    const char *a_sl, *a_exp, *a_offs, *a_pair, *a_space, *a_track, *a_sexp, *a_conn, *a_rsv, *a_closed;
    Py_ssize_t l_sl, l_exp, l_offs, l_pair, l_space, l_track, l_sexp, l_conn, l_rsv, l_closed;
    unsigned int n_pairs;
    if (!PyArg_ParseTuple(args, "Oy#y#O!y#y#y#y#y#Iy#y#y#", &t, &a_sl, &l_sl, &a_exp, &l_exp, &PyList_Type, &packets,
                          &a_offs, &l_offs, &a_pair, &l_pair, &a_space, &l_space, &a_track, &l_track, &a_sexp,
                          &l_sexp, &n_pairs, &a_conn, &l_conn, &a_rsv, &l_rsv, &a_closed, &l_closed))
        return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    const Py_ssize_t n = PyList_Size(packets);
    if (check_len(l_sl, n, 4, "slots") < 0 || check_len(l_exp, n, 8, "exp") < 0 ||
        check_len(l_offs, n, 4, "offs") < 0 || check_len(l_pair, n, 4, "pair") < 0 ||
        check_len(l_space, n, 4, "space") < 0 || check_len(l_track, n, 1, "track") < 0 ||
        check_len(l_conn, n, 4, "conn") < 0 || check_len(l_rsv, n, 1, "rsv") < 0 || l_sexp % 8)
        return l_sexp % 8 ? (PyErr_SetString(PyExc_ValueError, "space_exp: whole u64 items"), NULL) : NULL;
    const Py_ssize_t n_spaces = l_sexp / 8, n_conns = l_closed;
    const uint32_t *slots = (const uint32_t *)a_sl, *offs = (const uint32_t *)a_offs, *pair = (const uint32_t *)a_pair,
                   *space = (const uint32_t *)a_space, *conn = (const uint32_t *)a_conn;
    const uint64_t *exp = (const uint64_t *)a_exp;
    const uint8_t *track = (const uint8_t *)a_track, *rsv = (const uint8_t *)a_rsv;
    PyObject *ret = NULL, *outs = NULL, *res = NULL, *deferred = NULL, *sexp_out = NULL, *closed_out = NULL;
    qpp_desc *desc = NULL;
    uint8_t *blocked_pair = NULL, *blocked_space = NULL, *blocked_conn = NULL;
    sexp_out = PyBytes_FromStringAndSize(a_sexp, l_sexp);  /* the spaces' expected numbers, advanced below */
    closed_out = PyBytes_FromStringAndSize(a_closed, l_closed); /* the connections' closed flags, set below */
    if (!sexp_out || !closed_out) goto done;
    uint64_t *sx = (uint64_t *)PyBytes_AsString(sexp_out);
    uint8_t *closed = (uint8_t *)PyBytes_AsString(closed_out);
    for (Py_ssize_t i = 0; i < n; ++i)
        if (pair[i] >= n_pairs || (Py_ssize_t)space[i] >= n_spaces ||
            (conn[i] != WALK_NO_CONN && (Py_ssize_t)conn[i] >= n_conns)) {
            PyErr_SetString(PyExc_ValueError, "pair, space or connection index out of range");
            goto done;
        }
    /* sizes, then the launch over the session's pinned staging */
    size_t total = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *o = PyList_GetItem(packets, i);
        if (!PyBytes_Check(o)) {
            PyErr_SetString(PyExc_TypeError, "packets must be bytes");
            goto done;
        }
        total += (size_t)PyBytes_Size(o);
    }
    desc = (qpp_desc *)calloc(n ? (size_t)n : 1, sizeof(qpp_desc));
    res = PyBytes_FromStringAndSize(NULL, n * (Py_ssize_t)sizeof(qpp_result));
    blocked_pair = (uint8_t *)calloc(n_pairs ? n_pairs : 1, 1);
    blocked_space = (uint8_t *)calloc(n_spaces ? (size_t)n_spaces : 1, 1);
    blocked_conn = (uint8_t *)calloc(n_conns ? (size_t)n_conns : 1, 1);
    outs = PyList_New(n);
    deferred = PyList_New(0);
    if (!desc || !res || !blocked_pair || !blocked_space || !blocked_conn || !outs || !deferred) {
        PyErr_NoMemory();
        goto done;
    }
    uint8_t *hin = NULL, *hout = NULL;
    if (n) {
        qpp_session *s = session();
        if (!s || check_rc(qpp_session_stage(s, total ? total : 1, (uint32_t)n, &hin, &hout)) < 0) goto done;
        size_t off = 0;
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject *o = PyList_GetItem(packets, i);
            const size_t l = (size_t)PyBytes_Size(o);
            memcpy(hin + off, PyBytes_AsString(o), l);
            qpp_desc *d = &desc[i];
            d->in_off = d->out_off = off;
            d->len = (uint32_t)l;
            d->hdr_len = offs[i] > 0xffff ? 0xffff : (uint16_t)offs[i];
            d->pn = exp[i];
            d->slot = slots[i];
            off += l;
        }
        if (host_call(0, kt, desc, (uint32_t)n, hin, total, hout, total, PyBytes_AsString(res)) < 0) goto done;
    }
    {
        qpp_result *r = (qpp_result *)PyBytes_AsString(res);
        /* no receive key (crypto.py:78-79) and packet-number offsets past the
           header limit fail whatever the launch left in their results */
        for (Py_ssize_t i = 0; i < n; ++i) {
            if (slots[i] == 0xffffffffu) r[i].status = QPP_S_NO_KEY;
            else if (offs[i] > QPP_MAX_HDR) r[i].status = QPP_S_LENGTH;
        }
        for (Py_ssize_t i = 0; i < n; ++i) {
            const uint32_t p = pair[i], sp = space[i], c = conn[i];
            PyObject *item = Py_None;
            Py_INCREF(Py_None);
            PyList_SetItem(outs, i, item);
            int defer = blocked_pair[p] || blocked_space[sp] || (c != WALK_NO_CONN && blocked_conn[c]);
            if (!defer && c != WALK_NO_CONN && closed[c]) {
                r[i].status = WALK_S_CLOSED; /* connection.py:756-757 */
                continue;
            }
            const uint16_t st = r[i].status;
            const uint64_t now = sx[sp];
            if (!defer && st == QPP_S_KEY_PHASE) defer = 1;
            if (!defer && now != exp[i] && (st == QPP_S_OK || st == QPP_S_DECRYPT)) {
                const int pn_len = (int)r[i].hdr_len - (int)offs[i];
                if (pn_len < 1 || pn_len > 4 || decode_pn_signed(r[i].pn, pn_len, now) != (int64_t)r[i].pn) defer = 1;
            }
            if (defer) {
                blocked_pair[p] = blocked_space[sp] = 1;
                if (c != WALK_NO_CONN) blocked_conn[c] = 1;
                PyObject *ix = PyLong_FromSsize_t(i);
                if (!ix || PyList_Append(deferred, ix) < 0) {
                    Py_XDECREF(ix);
                    goto done;
                }
                Py_DECREF(ix);
                continue;
            }
            if (st != QPP_S_OK) continue;
            const uint8_t *o = hout + desc[i].out_off;
            if (rsv[i] && r[i].hdr_len && (o[0] & rsv[i])) {
                /* connection.py:949-960: close, end, no expected-number update */
                r[i].status = WALK_S_RESERVED;
                if (c != WALK_NO_CONN) closed[c] = 1;
                continue;
            }
            PyObject *h = PyBytes_FromStringAndSize((const char *)o, r[i].hdr_len);
            PyObject *pl = PyBytes_FromStringAndSize((const char *)o + r[i].hdr_len,
                                                     (Py_ssize_t)r[i].out_len - r[i].hdr_len);
            PyObject *pn = PyLong_FromUnsignedLongLong(r[i].pn);
            item = (h && pl && pn) ? PyTuple_Pack(3, h, pl, pn) : NULL;
            Py_XDECREF(h);
            Py_XDECREF(pl);
            Py_XDECREF(pn);
            if (!item) goto done;
            PyObject_GC_UnTrack(item); /* bytes and an int: never in a cycle (make_record) */
            PyList_SetItem(outs, i, item);
            if (track[i] && r[i].pn > now) sx[sp] = r[i].pn + 1;
        }
    }
    ret = PyTuple_Pack(5, outs, res, deferred, sexp_out, closed_out);
done:
    Py_XDECREF(sexp_out);
    Py_XDECREF(closed_out);
    Py_XDECREF(outs);
    Py_XDECREF(res);
    Py_XDECREF(deferred);
    free(desc);
    free(blocked_pair);
    free(blocked_space);
    free(blocked_conn);
    return ret;
}

/* ------------------------------------------ batched receive, short headers -- */

/* Identity map from object pointers to small indices (open addressing). */
typedef struct {
    const void **key;
    uint32_t *val;
    size_t cap;
} PtrMap;

static int ptrmap_init(PtrMap *m, size_t n)
{
    m->cap = 16;
    while (m->cap < 2 * n + 1) m->cap <<= 1;
    m->key = (const void **)calloc(m->cap, sizeof(void *));
    m->val = (uint32_t *)calloc(m->cap, sizeof(uint32_t));
    return m->key && m->val ? 0 : -1;
}

static void ptrmap_free(PtrMap *m)
{
    free(m->key);
    free(m->val);
}

/* index of k, or insert it with value v (returns the stored value) */
static uint32_t ptrmap_get(PtrMap *m, const void *k, uint32_t v, int *inserted)
{
    size_t h = ((uintptr_t)k >> 4) * 0x9E3779B97F4A7C15ull;
    for (size_t i = h & (m->cap - 1);; i = (i + 1) & (m->cap - 1)) {
        if (m->key[i] == k) {
            *inserted = 0;
            return m->val[i];
        }
        if (!m->key[i]) {
            m->key[i] = k;
            m->val[i] = v;
            *inserted = 1;
            return v;
        }
    }
}

/* first_of_each(items) -> the distinct first elements of the (a, b) tuples of
 * `items`, by identity, in first-seen order (the connections of a batch of
 * (connection, datagram) pairs). */
static PyObject *py_first_of_each(PyObject *m, PyObject *args)
{
    PyObject *items;
    if (!PyArg_ParseTuple(args, "O!", &PyList_Type, &items)) return NULL;
    const Py_ssize_t n = PyList_Size(items);
    PtrMap pm;
    if (ptrmap_init(&pm, 64) < 0) return PyErr_NoMemory();
    PyObject *out = PyList_New(0);
    for (Py_ssize_t i = 0; out && i < n; ++i) {
        PyObject *it = PyList_GetItem(items, i);
        PyObject *a = PyTuple_Check(it) && PyTuple_Size(it) == 2 ? PyTuple_GetItem(it, 0) : NULL;
        if (!a) {
            PyErr_SetString(PyExc_TypeError, "items must be (connection, datagram) tuples");
            Py_CLEAR(out);
            break;
        }
        int ins;
        if ((size_t)PyList_Size(out) * 2 + 2 > pm.cap) {
            /* grow: rebuild from the list */
            PtrMap g;
            if (ptrmap_init(&g, (size_t)PyList_Size(out) * 2 + 2) < 0) {
                Py_CLEAR(out);
                PyErr_NoMemory();
                break;
            }
            for (Py_ssize_t k = 0; k < PyList_Size(out); ++k) (void)ptrmap_get(&g, PyList_GetItem(out, k), (uint32_t)k, &ins);
            ptrmap_free(&pm);
            pm = g;
        }
        (void)ptrmap_get(&pm, a, (uint32_t)PyList_Size(out), &ins);
        if (ins && PyList_Append(out, a) < 0) Py_CLEAR(out);
    }
    ptrmap_free(&pm);
    return out;
}

/* A record of the caller's tuple subclass (receive.ReceivedPacket), built
 * without a Python-level call: fields are borrowed references.  A record
 * refers only to objects that cannot refer back to it (ints, bytes, None,
 * enum members), so it can never be part of a reference cycle: it is taken
 * off the cycle collector's lists, which a batch of 64 Ki records would
 * otherwise keep traversing. */
static PyObject *make_record(PyTypeObject *tp, allocfunc alloc, PyObject *const *f, int nf)
{
    PyObject *r = alloc(tp, nf);
    if (!r) return NULL;
    for (int k = 0; k < nf; ++k) {
        Py_INCREF(f[k]);
        if (PyTuple_SetItem(r, k, f[k]) < 0) {
            Py_DECREF(r);
            return NULL;
        }
    }
    PyObject_GC_UnTrack(r);
    return r;
}

/* receive_short(table, items, conns, conn_cid_u32, conn_pair_u32,
 *               conn_space_u32, pair_slot_u32, space_exp_u64, rec_type,
 *               packet_type, epoch, conn_closed_u8)
 *     -> None | (records, deferred, space_exp after, conn_closed after)
 * receive_datagrams' steady state in one call: every datagram of `items`
 * ((connection, bytes) pairs) is a short-header 1-RTT packet running to the
 * datagram's end (RFC 9000 sec. 12.2), its encrypted offset 1 + the
 * connection's CID length.  One launch, then the in-order walk of
 * CryptoPair.decrypt_packet (quic/crypto.py:184-192) with the expected
 * packet numbers of connection.py:984-985, as unprotect_walk does, and one
 * record per datagram:
 *   (datagram, 0, None, packet_type, epoch, plain_header, payload, pn, None),
 *   or the drop: "key_unavailable" (pair_slot 0xffffffff: no receive key,
 *   crypto.py:78-79) / "payload_decrypt_error" (connection.py:936-947) /
 *   "reserved_bits" (a packet that authenticates with a reserved bit set
 *   closes its connection, connection.py:949-960, and leaves the expected
 *   number alone) / "connection_closed" (epoch None: a datagram of a closed
 *   connection, ignored by connection.py:756-757; nothing is launched for the
 *   connections closed on entry).
 * Deferred datagrams (key-phase flip, or a number that decodes differently
 * by now -- and every later one of their pair, space or connection) get None and their
 * index in `deferred`, for the caller's general path.  Returns None at once,
 * with nothing launched, if any datagram is not such a packet. */
static PyObject *py_receive_short(PyObject *m, PyObject *args)
{
    PyObject *t, *items, *conns, *rec_type, *ptype, *epoch;
    const char *a_cid, *a_pair, *a_space, *a_pslot, *a_sexp, *a_closed;
    Py_ssize_t l_cid, l_pair, l_space, l_pslot, l_sexp, l_closed;
    if (!PyArg_ParseTuple(args, "OO!O!y#y#y#y#y#OOOy#", &t, &PyList_Type, &items, &PyList_Type, &conns, &a_cid,
                          &l_cid, &a_pair, &l_pair, &a_space, &l_space, &a_pslot, &l_pslot, &a_sexp, &l_sexp,
                          &rec_type, &ptype, &epoch, &a_closed, &l_closed))
        return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    if (!PyType_Check(rec_type) || !PyType_IsSubtype((PyTypeObject *)rec_type, &PyTuple_Type)) {
        PyErr_SetString(PyExc_TypeError, "rec_type must be a tuple subclass");
        return NULL;
    }
    const Py_ssize_t n = PyList_Size(items), nc = PyList_Size(conns);
    const Py_ssize_t n_pairs = l_pslot / 4, n_spaces = l_sexp / 8;
    if (check_len(l_cid, nc, 4, "conn_cid") < 0 || check_len(l_pair, nc, 4, "conn_pair") < 0 ||
        check_len(l_space, nc, 4, "conn_space") < 0 || check_len(l_closed, nc, 1, "conn_closed") < 0)
        return NULL;
    const uint32_t *ccid = (const uint32_t *)a_cid, *cpair = (const uint32_t *)a_pair,
                   *cspace = (const uint32_t *)a_space, *pslot = (const uint32_t *)a_pslot;
    for (Py_ssize_t c = 0; c < nc; ++c)
        if ((Py_ssize_t)cpair[c] >= n_pairs || (Py_ssize_t)cspace[c] >= n_spaces) {
            PyErr_SetString(PyExc_ValueError, "pair or space index out of range");
            return NULL;
        }
    PyTypeObject *tp = (PyTypeObject *)rec_type;
    allocfunc alloc = (allocfunc)PyType_GetSlot(tp, Py_tp_alloc);
    if (!alloc) return NULL;
    /* a snapshot holding a reference to every (connection, datagram) item:
       the datagram copies below run without the GIL, while another thread
       may change the caller's list */
    items = PySequence_Tuple(items);
    if (!items) return NULL;

    PtrMap pm = {0};
    uint32_t *conn_of = NULL, *slot_of = NULL;
    qpp_desc *desc = NULL;
    uint8_t **cd = NULL;
    const uint8_t **cs = NULL;
    size_t *cl = NULL;
    uint8_t *blocked_pair = NULL, *blocked_space = NULL, *blocked_conn = NULL;
    PyObject *ret = NULL, *recs = NULL, *res = NULL, *deferred = NULL, *sexp_out = NULL, *closed_out = NULL;
    PyObject *empty = NULL, *minus1 = NULL, *zero = NULL, *s_key = NULL, *s_dec = NULL, *s_rsv = NULL, *s_closed = NULL;
    uint8_t **od = NULL;
    const uint8_t **os_ = NULL;
    size_t *ol = NULL, on = 0, otot = 0;
    int ins;
    if (ptrmap_init(&pm, (size_t)nc) < 0) goto nomem;
    for (Py_ssize_t c = 0; c < nc; ++c) (void)ptrmap_get(&pm, PyList_GetItem(conns, c), (uint32_t)c, &ins);
    conn_of = (uint32_t *)malloc((n ? (size_t)n : 1) * sizeof(uint32_t));
    slot_of = (uint32_t *)malloc((n ? (size_t)n : 1) * sizeof(uint32_t));
    desc = (qpp_desc *)calloc(n ? (size_t)n : 1, sizeof(qpp_desc));
    cd = (uint8_t **)malloc((n ? (size_t)n : 1) * sizeof(uint8_t *));
    cs = (const uint8_t **)malloc((n ? (size_t)n : 1) * sizeof(uint8_t *));
    cl = (size_t *)malloc((n ? (size_t)n : 1) * sizeof(size_t));
    blocked_pair = (uint8_t *)calloc(n_pairs ? (size_t)n_pairs : 1, 1);
    blocked_space = (uint8_t *)calloc(n_spaces ? (size_t)n_spaces : 1, 1);
    blocked_conn = (uint8_t *)calloc(nc ? (size_t)nc : 1, 1);
    /* output copies: header and payload of every packet, filled after the
       walk without the GIL (the bytes objects are not shared until returned) */
    od = (uint8_t **)malloc((2 * (size_t)n + 1) * sizeof(uint8_t *));
    os_ = (const uint8_t **)malloc((2 * (size_t)n + 1) * sizeof(uint8_t *));
    ol = (size_t *)malloc((2 * (size_t)n + 1) * sizeof(size_t));
    if (!conn_of || !slot_of || !desc || !cd || !cs || !cl || !blocked_pair || !blocked_space || !blocked_conn || !od ||
        !os_ || !ol)
        goto nomem;
    /* classify: every datagram a short header long enough for its CID */
    size_t total = 0;
    uint32_t nl = 0;  /* packets to launch */
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *it = PyTuple_GetItem(items, i);
        PyObject *c = PyTuple_Check(it) && PyTuple_Size(it) == 2 ? PyTuple_GetItem(it, 0) : NULL;
        PyObject *d = c ? PyTuple_GetItem(it, 1) : NULL;
        if (!d || !PyBytes_Check(d)) goto fallback;
        const int found = (int)ptrmap_get(&pm, c, 0xffffffffu, &ins);
        if (ins) goto fallback; /* a connection not in conns */
        const Py_ssize_t len = PyBytes_Size(d);
        const uint8_t *b = (const uint8_t *)PyBytes_AsString(d);
        if (len < 1 || (b[0] & 0xC0) != 0x40 || len < 1 + (Py_ssize_t)ccid[found]) goto fallback;
        conn_of[i] = (uint32_t)found;
        slot_of[i] = ((const uint8_t *)a_closed)[found] ? RS_CLOSED : pslot[cpair[found]];
        if (slot_of[i] >= RS_CLOSED) continue; /* closed on entry, or no receive key: no launch */
        qpp_desc *x = &desc[nl];
        x->in_off = x->out_off = total;
        x->len = (uint32_t)len;
        x->hdr_len = (uint16_t)(1 + ccid[found]);
        x->pn = ((const uint64_t *)a_sexp)[cspace[found]];
        x->slot = slot_of[i];
        x->rsv = (uint32_t)i; /* the datagram (host-side bookkeeping only) */
        cs[nl] = b;
        cl[nl] = (size_t)len;
        total += (size_t)len;
        ++nl;
    }
    res = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)nl * (Py_ssize_t)sizeof(qpp_result));
    sexp_out = PyBytes_FromStringAndSize(a_sexp, l_sexp);
    closed_out = PyBytes_FromStringAndSize(a_closed, l_closed);
    recs = PyList_New(n);
    deferred = PyList_New(0);
    empty = PyBytes_FromStringAndSize("", 0);
    minus1 = PyLong_FromLong(-1);
    zero = PyLong_FromLong(0);
    s_key = PyUnicode_FromString("key_unavailable");
    s_dec = PyUnicode_FromString("payload_decrypt_error");
    s_rsv = PyUnicode_FromString("reserved_bits");
    s_closed = PyUnicode_FromString("connection_closed");
    if (!res || !sexp_out || !closed_out || !recs || !deferred || !empty || !minus1 || !zero || !s_key || !s_dec ||
        !s_rsv || !s_closed)
        goto nomem;
    uint8_t *hin = NULL, *hout = NULL;
    if (nl) {
        qpp_session *ss = session();
        if (!ss || check_rc(qpp_session_stage(ss, total ? total : 1, nl, &hin, &hout)) < 0) goto done;
        for (uint32_t k = 0; k < nl; ++k) cd[k] = hin + desc[k].in_off;
        Py_BEGIN_ALLOW_THREADS  /* the snapshot holds every datagram */
        par_copy(cd, cs, cl, nl, total);
        Py_END_ALLOW_THREADS
        if (host_call(0, kt, desc, nl, hin, total, hout, total, PyBytes_AsString(res)) < 0) goto done;
    }
    {
        uint64_t *sx = (uint64_t *)PyBytes_AsString(sexp_out);
        uint8_t *closed = (uint8_t *)PyBytes_AsString(closed_out);
        const qpp_result *r = (const qpp_result *)PyBytes_AsString(res);
        uint32_t k = 0;
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject *di = PyLong_FromSsize_t(i);
            if (!di) goto done;
            const uint32_t c = conn_of[i], p = cpair[c], sp = cspace[c];
            const int launched = slot_of[i] < RS_CLOSED;
            const qpp_result *ri = launched ? &r[k] : NULL;
            const qpp_desc *dk = launched ? &desc[k] : NULL;
            k += launched;
            /* a deferred packet of the connection may close it: wait for it */
            int defer = blocked_conn[c];
            if (!defer && launched) {
                const uint64_t now = sx[sp];
                defer = blocked_pair[p] || blocked_space[sp] || (!closed[c] && ri->status == QPP_S_KEY_PHASE);
                if (!defer && !closed[c] && now != dk->pn && (ri->status == QPP_S_OK || ri->status == QPP_S_DECRYPT)) {
                    const int pn_len = (int)ri->hdr_len - (int)dk->hdr_len;
                    if (pn_len < 1 || pn_len > 4 || decode_pn_signed(ri->pn, pn_len, now) != (int64_t)ri->pn)
                        defer = 1;
                }
            }
            if (defer) {
                blocked_conn[c] = 1;
                if (launched) blocked_pair[p] = blocked_space[sp] = 1;
                const int bad = PyList_Append(deferred, di);
                Py_INCREF(Py_None);
                PyList_SetItem(recs, i, Py_None);
                Py_DECREF(di);
                if (bad < 0) goto done;
                continue;
            }
            PyObject *rec = NULL;
            if (closed[c]) {
                /* connection.py:756-757 */
                PyObject *f[9] = {di, zero, Py_None, ptype, Py_None, empty, empty, minus1, s_closed};
                rec = make_record(tp, alloc, f, 9);
            } else if (!launched) {
                PyObject *f[9] = {di, zero, Py_None, ptype, epoch, empty, empty, minus1, s_key};
                rec = make_record(tp, alloc, f, 9);
            } else {
                const uint64_t now = sx[sp];
                if (ri->status == QPP_S_OK && (hout[dk->out_off] & 0x18)) {
                    /* connection.py:949-960: the close, before :984-985 */
                    closed[c] = 1;
                    PyObject *f[9] = {di, zero, Py_None, ptype, epoch, empty, empty, minus1, s_rsv};
                    rec = make_record(tp, alloc, f, 9);
                } else if (ri->status == QPP_S_OK) {
                    const uint8_t *o = hout + dk->out_off;
                    const size_t pll = (size_t)ri->out_len - ri->hdr_len;
                    PyObject *h = PyBytes_FromStringAndSize(NULL, ri->hdr_len);
                    PyObject *pl = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)pll);
                    PyObject *pn = PyLong_FromUnsignedLongLong(ri->pn);
                    if (h && pl && pn) {
                        od[on] = (uint8_t *)PyBytes_AsString(h), os_[on] = o, ol[on++] = ri->hdr_len;
                        od[on] = (uint8_t *)PyBytes_AsString(pl), os_[on] = o + ri->hdr_len, ol[on++] = pll;
                        otot += ri->hdr_len + pll;
                        PyObject *f[9] = {di, zero, Py_None, ptype, epoch, h, pl, pn, Py_None};
                        rec = make_record(tp, alloc, f, 9);
                    }
                    Py_XDECREF(h);
                    Py_XDECREF(pl);
                    Py_XDECREF(pn);
                    if (ri->pn > now) sx[sp] = ri->pn + 1;
                } else {
                    PyObject *f[9] = {di, zero, Py_None, ptype, epoch, empty, empty, minus1,
                                      ri->status == QPP_S_NO_KEY ? s_key : s_dec};
                    rec = make_record(tp, alloc, f, 9);
                }
            }
            Py_DECREF(di);
            if (!rec) goto done;
            PyList_SetItem(recs, i, rec);
        }
    }
    Py_BEGIN_ALLOW_THREADS
    par_copy(od, os_, ol, on, otot);
    Py_END_ALLOW_THREADS
    ret = PyTuple_Pack(4, recs, deferred, sexp_out, closed_out);
    goto done;
fallback:
    Py_INCREF(Py_None);
    ret = Py_None;
    goto done;
nomem:
    PyErr_NoMemory();
done:
    ptrmap_free(&pm);
    free(conn_of), free(slot_of), free(desc), free(cd), free(cs), free(cl), free(blocked_pair), free(blocked_space);
    free(blocked_conn), free(od), free(os_), free(ol);
    Py_DECREF(items);
    Py_XDECREF(closed_out);
    Py_XDECREF(s_rsv);
    Py_XDECREF(s_closed);
    Py_XDECREF(zero);
    Py_XDECREF(recs);
    Py_XDECREF(res);
    Py_XDECREF(deferred);
    Py_XDECREF(sexp_out);
    Py_XDECREF(empty);
    Py_XDECREF(minus1);
    Py_XDECREF(s_key);
    Py_XDECREF(s_dec);
    return ret;
}

static PyObject *py_hp_mask_host(PyObject *m, PyObject *args)
{
    PyObject *t;
    const char *slots, *samples;
    Py_ssize_t slots_len, samples_len;
    if (!PyArg_ParseTuple(args, "Oy#y#", &t, &slots, &slots_len, &samples, &samples_len))
        return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    uint32_t n = (uint32_t)(slots_len / 4);
    if (samples_len != (Py_ssize_t)n * 16) {
        PyErr_SetString(PyExc_ValueError, "need 16 sample bytes per slot");
        return NULL;
    }
    qpp_session *s = session();
    if (!s) return NULL;
    PyObject *out = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * 16);
    if (!out) return NULL;
    uint8_t *o = (uint8_t *)PyBytes_AsString(out);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_session_hp_mask(s, kt, (const uint32_t *)slots, (const uint8_t *)samples, n, o);
    Py_END_ALLOW_THREADS
    if (check_rc(rc) < 0) Py_CLEAR(out);
    return out;
}

static PyObject *py_device_ok(PyObject *m, PyObject *unused)
{
    return PyBool_FromLong(qpp_device_check() == QPP_OK);
}

static PyObject *py_abi(PyObject *m, PyObject *unused)
{
    return PyLong_FromLong(qpp_abi_version());
}

static PyObject *py_watchdog(PyObject *m, PyObject *unused)
{
    uint32_t v;
    Py_BEGIN_ALLOW_THREADS
    v = qpp_watchdog_count();
    Py_END_ALLOW_THREADS
    return PyLong_FromUnsignedLong(v);
}

#ifndef QPP_SOURCE_HASH
#error "build with -DQPP_SOURCE_HASH (aioquic_amd/build.py)"
#endif
/* the marker build.py reads back from the built extension */
static const char kSourceHash[] = "qpp-source-hash:" QPP_SOURCE_HASH;

static PyObject *py_source_hash(PyObject *m, PyObject *unused)
{
    return PyUnicode_FromString(kSourceHash + 16);
}

static PyMethodDef module_methods[] = {
    {"protect", py_protect, METH_VARARGS, "protect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream, plan=None)"},
    {"unprotect", py_unprotect, METH_VARARGS, "unprotect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream, plan=None)"},
    {"plan_build", py_plan_build, METH_VARARGS, "plan_build(plan, table, desc_ptr, n, stream)"},
    {"protect_host", py_protect_host, METH_VARARGS, "protect_host(table, desc, data, out_len) -> (out, results)"},
    {"unprotect_host", py_unprotect_host, METH_VARARGS, "unprotect_host(table, desc, data, out_len) -> (out, results)"},
    {"protect_into", py_protect_into, METH_VARARGS, "protect_into(table, desc_ptr, n, in_ptr, in_len, out_ptr, out_len, res_ptr)"},
    {"unprotect_into", py_unprotect_into, METH_VARARGS, "unprotect_into(table, desc_ptr, n, in_ptr, in_len, out_ptr, out_len, res_ptr)"},
    {"protect_list", py_protect_list, METH_VARARGS,
     "protect_list(table, slots_u32, pns_u64, headers, payloads) -> (wires, results)"},
    {"unprotect_list", py_unprotect_list, METH_VARARGS,
     "unprotect_list(table, slots_u32, expected_u64, packets, pn_offs_u32) -> (list of (header, payload) | None, results)"},
    {"protect_datagrams", py_protect_datagrams, METH_VARARGS,
     "protect_datagrams(table, plains, dg_u32, off_u32, hsize_u32, size_u32, pn_u64, slot_u32) -> (wires, results)"},
    {"unprotect_walk", py_unprotect_walk, METH_VARARGS,
     "unprotect_walk(table, slots_u32, exp_u64, packets, offs_u32, pair_u32, space_u32, track_u8, space_exp_u64, "
     "n_pairs, conn_u32, rsv_u8, closed_u8) -> (outcomes, results, deferred, space_exp, closed)"},
    {"first_of_each", py_first_of_each, METH_VARARGS, "first_of_each(items) -> distinct first elements, by identity"},
    {"receive_short", py_receive_short, METH_VARARGS,
     "receive_short(table, items, conns, conn_cid_u32, conn_pair_u32, conn_space_u32, pair_slot_u32, space_exp_u64, "
     "rec_type, packet_type, epoch) -> None | (records, deferred, space_exp)"},
    {"hp_mask_host", py_hp_mask_host, METH_VARARGS, "hp_mask_host(table, slots_u32, samples) -> masks"},
    {"device_ok", py_device_ok, METH_NOARGS, "True when a gfx950 device is usable"},
    {"abi_version", py_abi, METH_NOARGS, "C ABI version of libquicpp"},
    {"watchdog_count", py_watchdog, METH_NOARGS, "GCM table-entry watchdog events on the current device (0 expected)"},
    {"source_hash", py_source_hash, METH_NOARGS, "hash of the native sources this module was built from"},
    {NULL},
};

static struct PyModuleDef moduledef = {
    PyModuleDef_HEAD_INIT, "aioquic_amd._crypto", "GPU packet protection (libquicpp binding).",
    -1, module_methods,
};

static int add_type(PyObject *m, PyType_Spec *spec, const char *name, PyObject **slot)
{
    PyObject *t = PyType_FromSpec(spec);
    if (!t) return -1;
    *slot = t;
    Py_INCREF(t);
    return PyModule_AddObject(m, name, t);
}

/* Refuse a stale build: libquicpp.so and this extension must come from the
 * same sources, and those must be the tree's current ones (when present). */
static int check_sources(void)
{
    const char *mine = kSourceHash + 16, *lib = qpp_source_hash();
    if (strcmp(mine, lib) != 0) {
        PyErr_Format(PyExc_ImportError,
                     "aioquic_amd: libquicpp.so (sources %s) and _crypto (sources %s) come from different "
                     "builds; run python -m aioquic_amd.build", lib, mine);
        return -1;
    }
    PyObject *mod = PyImport_ImportModule("aioquic_amd._srchash");
    if (!mod) return -1;
    PyObject *tree = PyObject_CallMethod(mod, "tree_hash", NULL);
    Py_DECREF(mod);
    if (!tree) return -1;
    int rc = 0;
    if (tree != Py_None && PyUnicode_CompareWithASCIIString(tree, mine) != 0) {
        if (!PyErr_Occurred())
            PyErr_Format(PyExc_ImportError,
                         "aioquic_amd: the native sources (%S) changed since _crypto was built (%s); "
                         "run python -m aioquic_amd.build", tree, mine);
        rc = -1;
    }
    Py_DECREF(tree);
    return rc;
}

PyMODINIT_FUNC PyInit__crypto(void)
{
    if (check_sources() < 0) return NULL;
    PyObject *m = PyModule_Create(&moduledef);
    if (!m) return NULL;
    g_crypto_error = PyErr_NewException("aioquic_amd._crypto.CryptoError", PyExc_ValueError, NULL);
    if (!g_crypto_error) return NULL;
    Py_INCREF(g_crypto_error);
    if (PyModule_AddObject(m, "CryptoError", g_crypto_error) < 0) return NULL;
    if (add_type(m, &AEAD_spec, "AEAD", &g_aead_type) < 0 ||
        add_type(m, &HP_spec, "HeaderProtection", &g_hp_type) < 0 ||
        add_type(m, &KT_spec, "KeyTable", &g_kt_type) < 0 ||
        add_type(m, &Plan_spec, "Plan", &g_plan_type) < 0 ||
        add_type(m, &Multi_spec, "MultiSession", &g_multi_type) < 0)
        return NULL;
    PyModule_AddIntConstant(m, "DESC_SIZE", (long)sizeof(qpp_desc));
    PyModule_AddIntConstant(m, "RESULT_SIZE", (long)sizeof(qpp_result));
    PyModule_AddIntConstant(m, "KEY_MATERIAL_SIZE", (long)sizeof(qpp_key_material));
    return m;
}
