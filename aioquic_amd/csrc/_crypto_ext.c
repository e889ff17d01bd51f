/*
 * aioquic_amd._crypto -- CPython binding of libquicpp.so (include/quic_pp.h).
 *
 * Object API identical to the reference's aioquic._crypto (src/aioquic/_crypto.pyi:1-15):
 *   AEAD(cipher_name, key, iv).encrypt(data, associated_data, packet_number) -> bytes
 *                             .decrypt(data, associated_data, packet_number) -> bytes
 *   HeaderProtection(cipher_name, key).apply(plain_header, protected_payload) -> bytes
 *                                     .remove(packet, encrypted_offset) -> (bytes, int)
 *   CryptoError(ValueError), with the reference's messages (_crypto.c:17-29,79-90,126-152).
 * Every byte of crypto runs on the GPU through libquicpp; there is no CPU path.
 * Without a gfx950 device the constructors raise RuntimeError.
 *
 * Batch API (device pointers as ints, for torch tensors / the batch engine):
 *   KeyTable(capacity) .set(materials) .clear(slots) .capacity
 *   protect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream) -> None
 *   unprotect(...)                                                  -> None
 *   protect_host(table, desc, data, out_len) -> (bytes out, bytes results)
 *   unprotect_host(table, desc, data, out_len) -> (bytes out, bytes results)
 *   hp_mask_host(table, slots, samples) -> bytes
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <ctype.h>
#include <string.h>

#include "quic_pp.h"

static PyObject *g_crypto_error;
static qpp_session *g_session;

static qpp_session *session(void)
{
    if (!g_session) {
        int rc = qpp_session_create(1 << 16, 64, &g_session);
        if (rc != QPP_OK) {
            PyErr_Format(PyExc_RuntimeError, "aioquic_amd: cannot open a gfx950 session (%s)",
                         qpp_strerror(rc));
            return NULL;
        }
    }
    return g_session;
}

static int check_rc(int rc)
{
    if (rc == QPP_OK) return 0;
    PyErr_Format(PyExc_RuntimeError, "aioquic_amd: %s", qpp_strerror(rc));
    return -1;
}

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

/* ------------------------------------------------------------ key slot -- */

/* A single-slot device key table, created on first use. */
typedef struct {
    qpp_key_material km;
    qpp_keytab *kt;
} OneSlot;

static int oneslot_ready(OneSlot *o)
{
    if (o->kt) return 0;
    if (!session()) return -1;
    int rc = qpp_keytab_create(1, &o->kt);
    if (rc == QPP_OK) rc = qpp_session_set_keys(g_session, o->kt, &o->km, 1);
    if (rc != QPP_OK) {
        if (o->kt) qpp_keytab_destroy(o->kt);
        o->kt = NULL;
        return check_rc(rc);
    }
    return 0;
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
    if (self->s.kt) {
        qpp_keytab_destroy(self->s.kt);
        self->s.kt = NULL;
    }
    memset(&self->s.km, 0, sizeof(self->s.km));
    self->s.km.suite = (uint8_t)suite;
    memcpy(self->s.km.key, key, (size_t)key_len);
    memcpy(self->s.km.iv, iv, (size_t)iv_len); /* short iv: zero padded, as the reference */
    return oneslot_ready(&self->s);
}

static void AEAD_dealloc(AEADObject *self)
{
    if (self->s.kt) qpp_keytab_destroy(self->s.kt);
    Py_TYPE(self)->tp_free((PyObject *)self);
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
    int rc = enc ? qpp_session_protect(g_session, self->s.kt, &d, 1, buf, in_len, buf + in_len,
                                       out_len, &r)
                 : qpp_session_unprotect(g_session, self->s.kt, &d, 1, buf, in_len, buf + in_len,
                                         out_len, &r);
    PyObject *ret = NULL;
    if (check_rc(rc) == 0) {
        if (r.status == QPP_S_OK)
            ret = PyBytes_FromStringAndSize((const char *)buf + in_len + aad_len,
                                            enc ? data_len + QPP_TAG_LEN : data_len - QPP_TAG_LEN);
        else if (r.status == QPP_S_DECRYPT)
            PyErr_SetString(g_crypto_error, "Payload decryption failed");
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

static PyTypeObject AEADType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "aioquic_amd._crypto.AEAD",
    .tp_basicsize = sizeof(AEADObject),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "AEAD payload protection on the GPU",
    .tp_methods = AEAD_methods,
    .tp_init = (initproc)AEAD_init,
    .tp_new = PyType_GenericNew,
    .tp_dealloc = (destructor)AEAD_dealloc,
};

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
    if (self->s.kt) {
        qpp_keytab_destroy(self->s.kt);
        self->s.kt = NULL;
    }
    memset(&self->s.km, 0, sizeof(self->s.km));
    self->s.km.suite = (uint8_t)suite;
    memcpy(self->s.km.hp, key, (size_t)key_len);
    /* the AEAD half of the slot is unused by mask launches; give it a valid key */
    return oneslot_ready(&self->s);
}

static void HP_dealloc(HPObject *self)
{
    if (self->s.kt) qpp_keytab_destroy(self->s.kt);
    Py_TYPE(self)->tp_free((PyObject *)self);
}

static int hp_mask(HPObject *self, const unsigned char *sample, unsigned char mask[16])
{
    if (oneslot_ready(&self->s) < 0) return -1;
    uint32_t slot = 0;
    return check_rc(qpp_session_hp_mask(g_session, self->s.kt, &slot, sample, 1, mask));
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
    unsigned char *o = (unsigned char *)PyBytes_AS_STRING(out);
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

static PyTypeObject HPType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "aioquic_amd._crypto.HeaderProtection",
    .tp_basicsize = sizeof(HPObject),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "QUIC header protection masks on the GPU",
    .tp_methods = HP_methods,
    .tp_init = (initproc)HP_init,
    .tp_new = PyType_GenericNew,
    .tp_dealloc = (destructor)HP_dealloc,
};

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
    Py_TYPE(self)->tp_free((PyObject *)self);
}

/* set(materials: bytes-like of n packed qpp_key_material records, stream=0) */
static PyObject *KT_set(KeyTableObject *self, PyObject *args)
{
    Py_buffer b;
    unsigned long long stream = 0;
    if (!PyArg_ParseTuple(args, "y*|K", &b, &stream)) return NULL;
    if (b.len % (Py_ssize_t)sizeof(qpp_key_material)) {
        PyBuffer_Release(&b);
        PyErr_SetString(PyExc_ValueError, "materials must be a whole number of 84-byte records");
        return NULL;
    }
    uint32_t n = (uint32_t)(b.len / (Py_ssize_t)sizeof(qpp_key_material));
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_keytab_set(self->kt, (const qpp_key_material *)b.buf, n, (void *)(uintptr_t)stream);
    Py_END_ALLOW_THREADS
    PyBuffer_Release(&b);
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
    Py_buffer b;
    unsigned long long stream = 0;
    if (!PyArg_ParseTuple(args, "y*|K", &b, &stream)) return NULL;
    if (b.len % (Py_ssize_t)sizeof(qpp_secret)) {
        PyBuffer_Release(&b);
        PyErr_SetString(PyExc_ValueError, "secrets must be a whole number of 80-byte records");
        return NULL;
    }
    uint32_t n = (uint32_t)(b.len / (Py_ssize_t)sizeof(qpp_secret));
    PyObject *km = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * (Py_ssize_t)sizeof(qpp_key_material));
    if (!km) {
        PyBuffer_Release(&b);
        return NULL;
    }
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = qpp_keytab_derive(self->kt, (const qpp_secret *)b.buf, n,
                           (qpp_key_material *)PyBytes_AS_STRING(km), (void *)(uintptr_t)stream);
    Py_END_ALLOW_THREADS
    PyBuffer_Release(&b);
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
    Py_buffer b;
    if (!PyArg_ParseTuple(args, "y*", &b)) return NULL;
    int rc = qpp_keytab_clear(self->kt, (const uint32_t *)b.buf, (uint32_t)(b.len / 4), NULL);
    PyBuffer_Release(&b);
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

static PyTypeObject KTType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "aioquic_amd._crypto.KeyTable",
    .tp_basicsize = sizeof(KeyTableObject),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "device-resident expanded key slots",
    .tp_methods = KT_methods,
    .tp_getset = KT_getset,
    .tp_init = (initproc)KT_init,
    .tp_new = PyType_GenericNew,
    .tp_dealloc = (destructor)KT_dealloc,
};

static qpp_keytab *as_table(PyObject *o)
{
    if (!PyObject_TypeCheck(o, &KTType)) {
        PyErr_SetString(PyExc_TypeError, "expected a KeyTable");
        return NULL;
    }
    return ((KeyTableObject *)o)->kt;
}

/* -------------------------------------------------------- batch calls -- */

static PyObject *batch_dev(PyObject *args, int enc)
{
    PyObject *t;
    unsigned long long dp, ip, op, rp, sp;
    unsigned int n;
    if (!PyArg_ParseTuple(args, "OKIKKKK", &t, &dp, &n, &ip, &op, &rp, &sp)) return NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt) return NULL;
    int rc = enc ? qpp_protect(kt, (const qpp_desc *)(uintptr_t)dp, n, (const uint8_t *)(uintptr_t)ip,
                               (uint8_t *)(uintptr_t)op, (qpp_result *)(uintptr_t)rp, (void *)(uintptr_t)sp)
                 : qpp_unprotect(kt, (const qpp_desc *)(uintptr_t)dp, n, (const uint8_t *)(uintptr_t)ip,
                                 (uint8_t *)(uintptr_t)op, (qpp_result *)(uintptr_t)rp, (void *)(uintptr_t)sp);
    if (check_rc(rc) < 0) return NULL;
    Py_RETURN_NONE;
}

static PyObject *py_protect(PyObject *m, PyObject *args) { return batch_dev(args, 1); }
static PyObject *py_unprotect(PyObject *m, PyObject *args) { return batch_dev(args, 0); }

static PyObject *batch_host(PyObject *args, int enc)
{
    PyObject *t;
    Py_buffer desc, data;
    Py_ssize_t out_len;
    if (!PyArg_ParseTuple(args, "Oy*y*n", &t, &desc, &data, &out_len)) return NULL;
    PyObject *ret = NULL, *out = NULL, *res = NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt || !session()) goto done;
    if (desc.len % (Py_ssize_t)sizeof(qpp_desc) || out_len < 0) {
        PyErr_SetString(PyExc_ValueError, "bad descriptor buffer or output length");
        goto done;
    }
    uint32_t n = (uint32_t)(desc.len / (Py_ssize_t)sizeof(qpp_desc));
    out = PyBytes_FromStringAndSize(NULL, out_len);
    res = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * (Py_ssize_t)sizeof(qpp_result));
    if (!out || !res) goto done;
    /* the session writes every byte of out (zeros where no packet lands) for
       n > 0, so only an empty batch needs the zero fill here */
    if (n == 0) memset(PyBytes_AS_STRING(out), 0, (size_t)out_len);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = enc ? qpp_session_protect(g_session, kt, desc.buf, n, data.buf, (size_t)data.len,
                                   (uint8_t *)PyBytes_AS_STRING(out), (size_t)out_len,
                                   (qpp_result *)PyBytes_AS_STRING(res))
             : qpp_session_unprotect(g_session, kt, desc.buf, n, data.buf, (size_t)data.len,
                                     (uint8_t *)PyBytes_AS_STRING(out), (size_t)out_len,
                                     (qpp_result *)PyBytes_AS_STRING(res));
    Py_END_ALLOW_THREADS
    if (check_rc(rc) < 0) goto done;
    ret = PyTuple_Pack(2, out, res);
done:
    Py_XDECREF(out);
    Py_XDECREF(res);
    PyBuffer_Release(&desc);
    PyBuffer_Release(&data);
    return ret;
}

/* protect_into / unprotect_into(table, desc, data, out, results): the host
   form with caller-owned, writable output and result buffers (any buffer
   object, e.g. a numpy array reused across batches), so a large batch does
   not allocate and first-touch a fresh bytes object per call. */
static PyObject *batch_into(PyObject *args, int enc)
{
    PyObject *t;
    Py_buffer desc, data, out, res;
    if (!PyArg_ParseTuple(args, "Oy*y*w*w*", &t, &desc, &data, &out, &res)) return NULL;
    PyObject *ret = NULL;
    qpp_keytab *kt = as_table(t);
    if (!kt || !session()) goto done;
    if (desc.len % (Py_ssize_t)sizeof(qpp_desc)) {
        PyErr_SetString(PyExc_ValueError, "bad descriptor buffer");
        goto done;
    }
    uint32_t n = (uint32_t)(desc.len / (Py_ssize_t)sizeof(qpp_desc));
    if (res.len < (Py_ssize_t)n * (Py_ssize_t)sizeof(qpp_result)) {
        PyErr_SetString(PyExc_ValueError, "results buffer too small");
        goto done;
    }
    if (n == 0) memset(out.buf, 0, (size_t)out.len);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = enc ? qpp_session_protect(g_session, kt, desc.buf, n, data.buf, (size_t)data.len,
                                   (uint8_t *)out.buf, (size_t)out.len, (qpp_result *)res.buf)
             : qpp_session_unprotect(g_session, kt, desc.buf, n, data.buf, (size_t)data.len,
                                     (uint8_t *)out.buf, (size_t)out.len, (qpp_result *)res.buf);
    Py_END_ALLOW_THREADS
    if (check_rc(rc) < 0) goto done;
    ret = Py_None;
    Py_INCREF(ret);
done:
    PyBuffer_Release(&desc);
    PyBuffer_Release(&data);
    PyBuffer_Release(&out);
    PyBuffer_Release(&res);
    return ret;
}

static PyObject *py_protect_into(PyObject *m, PyObject *args) { return batch_into(args, 1); }
static PyObject *py_unprotect_into(PyObject *m, PyObject *args) { return batch_into(args, 0); }

static PyObject *py_protect_host(PyObject *m, PyObject *args) { return batch_host(args, 1); }
static PyObject *py_unprotect_host(PyObject *m, PyObject *args) { return batch_host(args, 0); }

static PyObject *py_hp_mask_host(PyObject *m, PyObject *args)
{
    PyObject *t;
    Py_buffer slots, samples;
    if (!PyArg_ParseTuple(args, "Oy*y*", &t, &slots, &samples)) return NULL;
    PyObject *out = NULL;
    qpp_keytab *kt = as_table(t);
    uint32_t n = (uint32_t)(slots.len / 4);
    if (kt && session()) {
        if (samples.len != (Py_ssize_t)n * 16) {
            PyErr_SetString(PyExc_ValueError, "need 16 sample bytes per slot");
        } else {
            out = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)n * 16);
            if (out && check_rc(qpp_session_hp_mask(g_session, kt, slots.buf, samples.buf, n,
                                                    (uint8_t *)PyBytes_AS_STRING(out))) < 0)
                Py_CLEAR(out);
        }
    }
    PyBuffer_Release(&slots);
    PyBuffer_Release(&samples);
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

static PyMethodDef module_methods[] = {
    {"protect", py_protect, METH_VARARGS, "protect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream)"},
    {"unprotect", py_unprotect, METH_VARARGS, "unprotect(table, desc_ptr, n, in_ptr, out_ptr, res_ptr, stream)"},
    {"protect_host", py_protect_host, METH_VARARGS, "protect_host(table, desc, data, out_len) -> (out, results)"},
    {"unprotect_host", py_unprotect_host, METH_VARARGS, "unprotect_host(table, desc, data, out_len) -> (out, results)"},
    {"protect_into", py_protect_into, METH_VARARGS, "protect_into(table, desc, data, out, results) -> None"},
    {"unprotect_into", py_unprotect_into, METH_VARARGS, "unprotect_into(table, desc, data, out, results) -> None"},
    {"hp_mask_host", py_hp_mask_host, METH_VARARGS, "hp_mask_host(table, slots_u32, samples) -> masks"},
    {"device_ok", py_device_ok, METH_NOARGS, "True when a gfx950 device is usable"},
    {"abi_version", py_abi, METH_NOARGS, "C ABI version of libquicpp"},
    {NULL},
};

static struct PyModuleDef moduledef = {
    PyModuleDef_HEAD_INIT, "aioquic_amd._crypto", "GPU packet protection (libquicpp binding).",
    -1, module_methods,
};

PyMODINIT_FUNC PyInit__crypto(void)
{
    PyObject *m = PyModule_Create(&moduledef);
    if (!m) return NULL;
    g_crypto_error = PyErr_NewException("aioquic_amd._crypto.CryptoError", PyExc_ValueError, NULL);
    if (!g_crypto_error || PyModule_AddObject(m, "CryptoError", g_crypto_error) < 0) return NULL;
    Py_INCREF(g_crypto_error);
    PyTypeObject *types[] = {&AEADType, &HPType, &KTType};
    const char *names[] = {"AEAD", "HeaderProtection", "KeyTable"};
    for (int i = 0; i < 3; ++i) {
        if (PyType_Ready(types[i]) < 0) return NULL;
        Py_INCREF(types[i]);
        if (PyModule_AddObject(m, names[i], (PyObject *)types[i]) < 0) return NULL;
    }
    PyModule_AddIntConstant(m, "DESC_SIZE", (long)sizeof(qpp_desc));
    PyModule_AddIntConstant(m, "RESULT_SIZE", (long)sizeof(qpp_result));
    PyModule_AddIntConstant(m, "KEY_MATERIAL_SIZE", (long)sizeof(qpp_key_material));
    return m;
}
