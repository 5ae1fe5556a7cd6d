// smx_host.cpp — native host side of the drop-in compose_oplogs: List[Op] -> SoA
// (marshal) and device results -> fresh Op objects (materialise).
//
// This is the CPython-object half of the boundary: it reads the
// same attributes, in the same order, with the same coercions as the reference composer
// (semmerge/compose.py:16-18 sort key, :64-82 chain values, :30-49 materialize,
// :117-127 _clone_op), and marshal.py / materialize.py restate it in Python line by line
// (they are the readable spec and the tests' cross-check).  Exceptions raised by user
// objects propagate unchanged.
//
// deepcopy: params / guards / effects / provenance are copied by a native walk when they
// are JSON-shaped trees (exact dict / list containers, each reached once; exact str /
// int / float / bool / None leaves, which copy.deepcopy returns as themselves); anything
// else — subclasses, tuples, shared or cyclic containers, other objects — goes to
// copy.deepcopy itself, so the result is always what deepcopy returns.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Names {
  PyObject *type, *provenance, *id, *target, *symbolId, *addressId, *params, *guards, *effects,
      *schemaVersion, *get, *timestamp, *newName, *newAddress, *newFile, *file, *renameContext;
  PyObject* empty;      // ()
  PyObject* kw_op;      // ("id", "schemaVersion", "type", "target", "params", "guards", "effects", "provenance")
  PyObject* kw_target;  // ("symbolId", "addressId")
};
Names N;

bool init_names() {
#define NM(f) if (!(N.f = PyUnicode_InternFromString(#f))) return false
  NM(type); NM(provenance); NM(id); NM(target); NM(symbolId); NM(addressId); NM(params);
  NM(guards); NM(effects); NM(schemaVersion); NM(get); NM(timestamp); NM(newName);
  NM(newAddress); NM(newFile); NM(file); NM(renameContext);
#undef NM
  N.kw_op = PyTuple_Pack(8, N.id, N.schemaVersion, N.type, N.target, N.params, N.guards, N.effects,
                         N.provenance);
  N.kw_target = PyTuple_Pack(2, N.symbolId, N.addressId);
  N.empty = PyTuple_New(0);
  return N.kw_op && N.kw_target && N.empty;
}

// Owned reference holder.
struct Ref {
  PyObject* p = nullptr;
  Ref() = default;
  explicit Ref(PyObject* q) : p(q) {}
  Ref(const Ref&) = delete;
  Ref& operator=(const Ref&) = delete;
  ~Ref() { Py_XDECREF(p); }
  void reset(PyObject* q) { Py_XDECREF(p); p = q; }
  PyObject* release() { PyObject* q = p; p = nullptr; return q; }
  explicit operator bool() const { return p != nullptr; }
};

struct Buf {
  Py_buffer v{};
  bool held = false;
  ~Buf() { if (held) PyBuffer_Release(&v); }
};

bool get_buf(PyObject* o, Buf& b, Py_ssize_t itemsize, Py_ssize_t n, bool writable, const char* what) {
  if (PyObject_GetBuffer(o, &b.v, (writable ? PyBUF_WRITABLE : 0) | PyBUF_C_CONTIGUOUS) < 0) return false;
  b.held = true;
  if (b.v.itemsize != itemsize || b.v.len < n * itemsize) {
    PyErr_Format(PyExc_ValueError, "%s: need %zd contiguous items of %zd bytes", what, n, itemsize);
    return false;
  }
  return true;
}

// mapping.get(key, dflt) with the dict fast path (new reference).
PyObject* map_get(PyObject* m, PyObject* key, PyObject* dflt) {
  if (PyDict_CheckExact(m)) {
    PyObject* v = PyDict_GetItemWithError(m, key);
    if (v) { Py_INCREF(v); return v; }
    if (PyErr_Occurred()) return nullptr;
    Py_INCREF(dflt);
    return dflt;
  }
  return PyObject_CallMethodObjArgs(m, N.get, key, dflt, nullptr);
}

// ---------------------------------------------------------------- key encodings (marshal.py)

// ISO-8601 "YYYY-MM-DDTHH:MM:SS[.fff]Z" -> int(YYYYMMDDhhmmss) * 2000 + (2*fff | 1999).
bool iso_key(PyObject* s, uint64_t* out) {
  if (PyUnicode_READY(s) < 0) {
    PyErr_Clear();
    return false;
  }
  if (PyUnicode_KIND(s) != PyUnicode_1BYTE_KIND) return false;
  const Py_ssize_t n = PyUnicode_GET_LENGTH(s);
  if (n != 20 && n != 24) return false;
  const unsigned char* c = PyUnicode_1BYTE_DATA(s);
  static const char pat[] = "dddd-dd-ddTdd:dd:dd";
  uint64_t whole = 0;
  for (int i = 0; i < 19; ++i) {
    if (pat[i] == 'd') {
      if (c[i] < '0' || c[i] > '9') return false;
      whole = whole * 10 + (c[i] - '0');
    } else if (c[i] != (unsigned char)pat[i]) {
      return false;
    }
  }
  uint64_t frac = 1999;
  if (n == 24) {
    if (c[19] != '.') return false;
    uint64_t f = 0;
    for (int i = 20; i < 23; ++i) {
      if (c[i] < '0' || c[i] > '9') return false;
      f = f * 10 + (c[i] - '0');
    }
    frac = 2 * f;
  }
  if (c[n - 1] != 'Z') return false;
  *out = whole * 2000 + frac;
  return true;
}

int hexval(unsigned char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  return -1;
}

// Canonical lowercase UUID (exact str) -> 128-bit value.
bool uuid_key(PyObject* s, uint64_t* hi, uint64_t* lo) {
  if (!PyUnicode_CheckExact(s)) return false;
  if (PyUnicode_READY(s) < 0) {
    PyErr_Clear();
    return false;
  }
  if (PyUnicode_KIND(s) != PyUnicode_1BYTE_KIND || PyUnicode_GET_LENGTH(s) != 36) return false;
  const unsigned char* c = PyUnicode_1BYTE_DATA(s);
  uint64_t h = 0, l = 0;
  int nd = 0;
  for (int i = 0; i < 36; ++i) {
    if (i == 8 || i == 13 || i == 18 || i == 23) {
      if (c[i] != '-') return false;
      continue;
    }
    const int v = hexval(c[i]);
    if (v < 0) return false;
    if (nd < 16) h = (h << 4) | (uint64_t)v;
    else l = (l << 4) | (uint64_t)v;
    ++nd;
  }
  *hi = h;
  *lo = l;
  return true;
}

// str of <= 15 UTF-8 bytes -> bytes zero padded + length byte, big endian halves.
// Returns 1 packed, 0 not packable, -1 needs the Python encoder (lone surrogates).
int packed_key(PyObject* s, uint64_t* hi, uint64_t* lo) {
  if (!PyUnicode_Check(s)) return 0;
  Py_ssize_t len = 0;
  const char* u = PyUnicode_AsUTF8AndSize(s, &len);
  if (!u) {
    PyErr_Clear();
    return -1;
  }
  if (len > 15) return 0;
  unsigned char b[16] = {0};
  std::memcpy(b, u, (size_t)len);
  b[15] = (unsigned char)len;
  uint64_t h = 0, l = 0;
  for (int i = 0; i < 8; ++i) h = (h << 8) | b[i];
  for (int i = 8; i < 16; ++i) l = (l << 8) | b[i];
  *hi = h;
  *lo = l;
  return 1;
}

struct Interner {  // value -> dense id, first-seen order
  PyObject* map = nullptr;
  PyObject* list = nullptr;  // optional: keeps the values in id order
  long long next = 0;        // ids handed out (fresh() ones included)
  ~Interner() { Py_XDECREF(map); Py_XDECREF(list); }
  bool init(bool keep_list) {
    map = PyDict_New();
    if (keep_list) list = PyList_New(0);
    return map && (!keep_list || list);
  }
  long long operator()(PyObject* key) {  // -1 on error
    PyObject* got = PyDict_GetItemWithError(map, key);
    if (got) return PyLong_AsLongLong(got);
    if (PyErr_Occurred()) return -1;
    const long long id = next++;
    Ref v(PyLong_FromLongLong(id));
    if (!v || PyDict_SetItem(map, key, v.p) < 0) return -1;
    if (list && PyList_Append(list, key) < 0) return -1;
    return id;
  }
  long long fresh() { return next++; }
};

// ---------------------------------------------------------------- marshal

// marshal_ops(ops, kind_rank, unknown, kmove, krename, default_ts, eq_key,
//             kind, ts, hi, lo, sym, v0, v1)
//   -> (n_sym, strings, ts_ok, id_mode, ts_strs | None, ids | None)
// ts_ok False: ts_strs holds every timestamp string for the rank encoder.
// id_mode 0 UUID, 1 packed, -1: ids holds every id for the Python encoder.
PyObject* marshal_ops(PyObject*, PyObject* args) {
  PyObject *ops, *kind_rank, *default_ts, *eq_key;
  int unknown, kmove, krename;
  PyObject *okind, *ots, *ohi, *olo, *osym, *ov0, *ov1;
  if (!PyArg_ParseTuple(args, "O!O!iiiUOOOOOOOO", &PyList_Type, &ops, &PyDict_Type, &kind_rank, &unknown,
                        &kmove, &krename, &default_ts, &eq_key, &okind, &ots, &ohi, &olo, &osym, &ov0, &ov1))
    return nullptr;
  const Py_ssize_t n = PyList_GET_SIZE(ops);
  Buf bk, bts, bhi, blo, bsym, bv0, bv1;
  if (!get_buf(okind, bk, 1, n, true, "kind") || !get_buf(ots, bts, 8, n, true, "ts") ||
      !get_buf(ohi, bhi, 8, n, true, "oid_hi") || !get_buf(olo, blo, 8, n, true, "oid_lo") ||
      !get_buf(osym, bsym, 4, n, true, "sym") || !get_buf(ov0, bv0, 4, n, true, "v0") ||
      !get_buf(ov1, bv1, 4, n, true, "v1"))
    return nullptr;
  auto* kind = (uint8_t*)bk.v.buf;
  auto* ts = (uint64_t*)bts.v.buf;
  auto* hi = (uint64_t*)bhi.v.buf;
  auto* lo = (uint64_t*)blo.v.buf;
  auto* sym = (uint32_t*)bsym.v.buf;
  auto* v0 = (int32_t*)bv0.v.buf;
  auto* v1 = (int32_t*)bv1.v.buf;

  Interner syms, strings, eq;
  if (!syms.init(false) || !strings.init(true) || !eq.init(false)) return nullptr;
  Ref ts_list(PyList_New(n)), id_list(PyList_New(n));
  if (!ts_list || !id_list) return nullptr;
  bool ts_ok = true, all_uuid = true;

  auto sid = [&](PyObject* v, int32_t* dst) -> bool {  // strings[str(v)]
    Ref s(PyObject_Str(v));
    if (!s) return false;
    const long long id = strings(s.p);
    if (id < 0) return false;
    *dst = (int32_t)id;
    return true;
  };

  for (Py_ssize_t k = 0; k < n; ++k) {
    PyObject* op = PyList_GET_ITEM(ops, k);
    // precedence.get(op.type, 99) (compose.py:18)
    Ref type(PyObject_GetAttr(op, N.type));
    if (!type) return nullptr;
    PyObject* r = PyDict_GetItemWithError(kind_rank, type.p);
    if (!r && PyErr_Occurred()) return nullptr;
    const int kr = r ? (int)PyLong_AsLong(r) : unknown;
    kind[k] = (uint8_t)kr;
    // str(op.provenance.get("timestamp", "1970-01-01T00:00:00Z")) (compose.py:17)
    Ref prov(PyObject_GetAttr(op, N.provenance));
    if (!prov) return nullptr;
    Ref tso(map_get(prov.p, N.timestamp, default_ts));
    if (!tso) return nullptr;
    PyObject* tss = PyObject_Str(tso.p);
    if (!tss) return nullptr;
    PyList_SET_ITEM(ts_list.p, k, tss);
    if (ts_ok && !iso_key(tss, &ts[k])) ts_ok = false;
    // op.id (compose.py:18)
    PyObject* id = PyObject_GetAttr(op, N.id);
    if (!id) return nullptr;
    PyList_SET_ITEM(id_list.p, k, id);
    if (all_uuid && !uuid_key(id, &hi[k], &lo[k])) all_uuid = false;
    // target.symbolId: dict key / == (compose.py:33,64)
    Ref tgt(PyObject_GetAttr(op, N.target));
    if (!tgt) return nullptr;
    Ref s(PyObject_GetAttr(tgt.p, N.symbolId));
    if (!s) return nullptr;
    const long long si = syms(s.p);
    if (si < 0) return nullptr;
    sym[k] = (uint32_t)si;
    v0[k] = -1;
    v1[k] = -1;
    if (kr != kmove && kr != krename) continue;
    Ref params(PyObject_GetAttr(op, N.params));
    if (!params) return nullptr;
    if (kr == krename) {  // newName: '!=' class (compose.py:66) and str(newName) (compose.py:72)
      Ref name(map_get(params.p, N.newName, Py_None));
      if (!name) return nullptr;
      bool nan = false;
      if (PyFloat_CheckExact(name.p)) {
        nan = std::isnan(PyFloat_AS_DOUBLE(name.p));
      } else if (PyFloat_Check(name.p)) {
        const int ne = PyObject_RichCompareBool(name.p, name.p, Py_NE);
        if (ne < 0) return nullptr;
        nan = ne == 1;
      }
      if (nan) {
        v0[k] = (int32_t)eq.fresh();  // NaN != NaN: a class of its own (marshal._EqClasses)
      } else {
        Ref key;
        if (PyUnicode_Check(name.p) || PyLong_Check(name.p) || PyFloat_Check(name.p) || name.p == Py_None) {
          Py_INCREF(name.p);
          key.reset(name.p);
        } else {
          key.reset(PyObject_CallOneArg(eq_key, name.p));
          if (!key) return nullptr;
        }
        const long long c = eq(key.p);
        if (c < 0) return nullptr;
        v0[k] = (int32_t)c;
      }
      if (!sid(name.p, &v1[k])) return nullptr;
    } else {  // moves: str(newAddress), str(newFile or file) (compose.py:75-82)
      Ref addr(map_get(params.p, N.newAddress, Py_None));
      if (!addr) return nullptr;
      if (addr.p != Py_None && !sid(addr.p, &v0[k])) return nullptr;
      Ref nfile(map_get(params.p, N.newFile, Py_None));
      if (!nfile) return nullptr;
      const int truthy = PyObject_IsTrue(nfile.p);
      if (truthy < 0) return nullptr;
      if (!truthy) {
        nfile.reset(map_get(params.p, N.file, Py_None));
        if (!nfile) return nullptr;
      }
      if (nfile.p != Py_None && !sid(nfile.p, &v1[k])) return nullptr;
    }
  }

  int id_mode = 0;
  if (!all_uuid) {
    id_mode = 1;
    for (Py_ssize_t k = 0; k < n && id_mode == 1; ++k) {
      const int p = packed_key(PyList_GET_ITEM(id_list.p, k), &hi[k], &lo[k]);
      if (p != 1) id_mode = -1;
    }
  }
  const Py_ssize_t n_sym = PyDict_GET_SIZE(syms.map);
  return Py_BuildValue("nOOiOO", n_sym, strings.list, ts_ok ? Py_True : Py_False, id_mode,
                       ts_ok ? Py_None : ts_list.p, id_mode >= 0 ? Py_None : id_list.p);
}

// ---------------------------------------------------------------- deepcopy of JSON trees

bool is_atom(PyObject* x) {
  return PyUnicode_CheckExact(x) || PyLong_CheckExact(x) || PyFloat_CheckExact(x) || PyBool_Check(x) ||
         x == Py_None;
}

// Copy of a tree of exact dicts / lists over atoms; nullptr + *tree=false when x is
// not such a tree (seen: containers reached so far — a second visit means sharing).
PyObject* copy_tree(PyObject* x, std::vector<PyObject*>& seen, bool* tree, int depth) {
  if (is_atom(x)) {
    Py_INCREF(x);
    return x;
  }
  const bool d = PyDict_CheckExact(x), l = PyList_CheckExact(x);
  if ((!d && !l) || depth > 64) {
    *tree = false;
    return nullptr;
  }
  for (PyObject* q : seen)
    if (q == x) {
      *tree = false;
      return nullptr;
    }
  seen.push_back(x);
  if (d) {
    {  // flat dict of atoms (the usual params / provenance): one table copy
      Py_ssize_t pos = 0;
      PyObject *key, *val;
      bool flat = true;
      while (flat && PyDict_Next(x, &pos, &key, &val)) flat = is_atom(key) && is_atom(val);
      if (flat) return PyDict_Copy(x);
    }
    Ref y(PyDict_New());
    if (!y) return nullptr;
    Py_ssize_t pos = 0;
    PyObject *key, *val;
    while (PyDict_Next(x, &pos, &key, &val)) {
      if (!is_atom(key)) {
        *tree = false;
        return nullptr;
      }
      Ref v(copy_tree(val, seen, tree, depth + 1));
      if (!v) return nullptr;
      if (PyDict_SetItem(y.p, key, v.p) < 0) return nullptr;
    }
    return y.release();
  }
  Ref y(PyList_New(0));
  if (!y) return nullptr;
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(x); ++i) {
    Ref v(copy_tree(PyList_GET_ITEM(x, i), seen, tree, depth + 1));
    if (!v) return nullptr;
    if (PyList_Append(y.p, v.p) < 0) return nullptr;
  }
  return y.release();
}

PyObject* deep_copy(PyObject* x, PyObject* deepcopy) {
  if (PyDict_CheckExact(x) && PyDict_GET_SIZE(x) == 0) return PyDict_New();
  std::vector<PyObject*> seen;
  bool tree = true;
  PyObject* y = copy_tree(x, seen, &tree, 0);
  if (y || tree) return y;  // copied, or a real error

  return PyObject_CallOneArg(deepcopy, x);
}

PyObject* py_deep_copy(PyObject*, PyObject* args) {
  PyObject *x, *deepcopy;
  if (!PyArg_ParseTuple(args, "OO", &x, &deepcopy)) return nullptr;
  return deep_copy(x, deepcopy);
}

// ---------------------------------------------------------------- materialise

// cls(**dict(zip(names, args))).  A plain dataclass — generated __init__ taking
// exactly `names`, object.__new__, no __post_init__ (smx_host_ctor_mode in
// materialize.py decides, once per class) — is built as its __init__ would build it:
// object.__new__(cls), then one setattr per field in order (object.__setattr__ when
// frozen).  Any other class is called.
struct Ctor {
  PyObject* mode_fn = nullptr;  // (cls, names) -> 0 call, 1 setattr, 2 object.__setattr__
  std::vector<std::pair<PyTypeObject*, int>> seen;
  int mode(PyTypeObject* cls, PyObject* names) {
    for (auto& e : seen)
      if (e.first == cls) return e.second;
    Ref r(PyObject_CallFunctionObjArgs(mode_fn, (PyObject*)cls, names, nullptr));
    if (!r) return -1;
    const int m = (int)PyLong_AsLong(r.p);
    if (m < 0 && PyErr_Occurred()) return -1;
    seen.emplace_back(cls, m);
    return m;
  }
  PyObject* make(PyTypeObject* cls, PyObject* const* args, PyObject* names) {
    const int m = mode(cls, names);
    if (m < 0) return nullptr;
    if (m == 0) return PyObject_Vectorcall((PyObject*)cls, args, 0, names);
    Ref obj(PyBaseObject_Type.tp_new(cls, N.empty, nullptr));
    if (!obj) return nullptr;
    for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(names); ++i) {
      PyObject* nm = PyTuple_GET_ITEM(names, i);
      const int rc = m == 1 ? PyObject_SetAttr(obj.p, nm, args[i]) : PyObject_GenericSetAttr(obj.p, nm, args[i]);
      if (rc < 0) return nullptr;
    }
    return obj.release();
  }
};

// Pauses the cyclic GC while building millions of acyclic objects (the collector
// would otherwise rescan the growing output); restores the caller's setting.
struct GcPause {
  int was;
  GcPause() : was(PyGC_Disable()) {}
  ~GcPause() {
    if (was) PyGC_Enable();
  }
};

PyObject* make_target(Ctor& ctor, PyTypeObject* tcls, PyObject* sym, PyObject* addr) {
  PyObject* a[2] = {sym, addr};
  return ctor.make(tcls, a, N.kw_target);
}

// materialize_ops(ops, kind, strings, order, addr, file, ctx, kmove, krename, deepcopy, ctor_mode)
// -> List[Op] (materialize.py; compose.py:30-49 on a compose.py:117-127 clone)
PyObject* materialize_ops(PyObject*, PyObject* args) {
  PyObject *ops, *strings, *deepcopy;
  PyObject *okind, *oorder, *oaddr, *ofile, *octx;
  int kmove, krename;
  Ctor ctor;
  if (!PyArg_ParseTuple(args, "O!OO!OOOOiiOO", &PyList_Type, &ops, &okind, &PyList_Type, &strings, &oorder,
                        &oaddr, &ofile, &octx, &kmove, &krename, &deepcopy, &ctor.mode_fn))
    return nullptr;
  GcPause gc_pause;
  const Py_ssize_t n_ops = PyList_GET_SIZE(ops), n_str = PyList_GET_SIZE(strings);
  Buf bk, bo, ba, bf, bc;
  if (!get_buf(okind, bk, 1, n_ops, false, "kind") || !get_buf(oorder, bo, 4, 0, false, "order")) return nullptr;
  const Py_ssize_t m = bo.v.len / 4;
  if (!get_buf(oaddr, ba, 4, m, false, "addr") || !get_buf(ofile, bf, 4, m, false, "file") ||
      !get_buf(octx, bc, 4, m, false, "ctx"))
    return nullptr;
  const auto* kind = (const uint8_t*)bk.v.buf;
  const auto* order = (const int32_t*)bo.v.buf;
  const auto* addr = (const int32_t*)ba.v.buf;
  const auto* file = (const int32_t*)bf.v.buf;
  const auto* ctx = (const int32_t*)bc.v.buf;
  auto str_at = [&](int32_t i) -> PyObject* {
    if (i >= n_str) {
      PyErr_SetString(PyExc_IndexError, "string id out of range");
      return nullptr;
    }
    return PyList_GET_ITEM(strings, i);
  };

  Ref out(PyList_New(m));
  if (!out) return nullptr;
  for (Py_ssize_t t = 0; t < m; ++t) {
    const int32_t src = order[t];
    if (src < 0 || src >= n_ops) {
      PyErr_SetString(PyExc_IndexError, "source index out of range");
      return nullptr;
    }
    PyObject* op = PyList_GET_ITEM(ops, src);
    Ref tgt(PyObject_GetAttr(op, N.target));
    if (!tgt) return nullptr;
    PyTypeObject* tcls = Py_TYPE(tgt.p);
    Ref id(PyObject_GetAttr(op, N.id)), sv, ty, tsym, taddr, ntgt, p, g, e, pr;
    if (!id || !(sv.reset(PyObject_GetAttr(op, N.schemaVersion)), sv) ||
        !(ty.reset(PyObject_GetAttr(op, N.type)), ty) || !(tsym.reset(PyObject_GetAttr(tgt.p, N.symbolId)), tsym) ||
        !(taddr.reset(PyObject_GetAttr(tgt.p, N.addressId)), taddr) ||
        !(ntgt.reset(make_target(ctor, tcls, tsym.p, taddr.p)), ntgt))
      return nullptr;
    {
      Ref x(PyObject_GetAttr(op, N.params));
      if (!x || !(p.reset(deep_copy(x.p, deepcopy)), p)) return nullptr;
      x.reset(PyObject_GetAttr(op, N.guards));
      if (!x || !(g.reset(deep_copy(x.p, deepcopy)), g)) return nullptr;
      x.reset(PyObject_GetAttr(op, N.effects));
      if (!x || !(e.reset(deep_copy(x.p, deepcopy)), e)) return nullptr;
      x.reset(PyObject_GetAttr(op, N.provenance));
      if (!x || !(pr.reset(deep_copy(x.p, deepcopy)), pr)) return nullptr;
    }
    PyObject* a8[8] = {id.p, sv.p, ty.p, ntgt.p, p.p, g.p, e.p, pr.p};
    Ref clone(ctor.make(Py_TYPE(op), a8, N.kw_op));
    if (!clone) return nullptr;

    const int k = kind[src];
    const int32_t a = addr[t], f = file[t], c = ctx[t];
    if (k == kmove) {
      if (a >= 0 || f >= 0) {
        Ref cp(PyObject_GetAttr(clone.p, N.params));
        if (!cp) return nullptr;
        PyObject* s;
        if (a >= 0 && (!(s = str_at(a)) || PyObject_SetItem(cp.p, N.newAddress, s) < 0)) return nullptr;
        if (f >= 0 && (!(s = str_at(f)) || PyObject_SetItem(cp.p, N.newFile, s) < 0)) return nullptr;
      }
    }
    if (a >= 0) {
      PyObject* s = str_at(a);
      if (!s) return nullptr;
      Ref nt(make_target(ctor, tcls, tsym.p, s));
      if (!nt || PyObject_SetAttr(clone.p, N.target, nt.p) < 0) return nullptr;
    }
    if (k == krename && f >= 0) {
      PyObject* s = str_at(f);
      Ref cp(PyObject_GetAttr(clone.p, N.params));
      if (!s || !cp || PyObject_SetItem(cp.p, N.newFile, s) < 0 || PyObject_SetItem(cp.p, N.file, s) < 0)
        return nullptr;
    }
    if (c >= 0 && k != krename) {  // {**params, "renameContext": ...}
      PyObject* s = str_at(c);
      Ref cp(PyObject_GetAttr(clone.p, N.params));
      if (!s || !cp) return nullptr;
      Ref nd(PyDict_New());
      if (!nd || PyDict_Update(nd.p, cp.p) < 0 || PyDict_SetItem(nd.p, N.renameContext, s) < 0 ||
          PyObject_SetAttr(clone.p, N.params, nd.p) < 0)
        return nullptr;
    }
    PyList_SET_ITEM(out.p, t, clone.release());
  }
  return out.release();
}

// ---------------------------------------------------------------- Op.from_dict

// dict(x) (new reference): a copy of an exact dict, else the dict constructor.
PyObject* dict_of(PyObject* x) {
  if (PyDict_CheckExact(x)) return PyDict_Copy(x);
  return PyObject_CallOneArg((PyObject*)&PyDict_Type, x);
}

// ops_from_dicts(items, op_cls, target_cls, ctor_mode) -> List[Op]: Op.from_dict of every
// item (ops.py:89-100), in the same evaluation order and with the same coercions:
//   id=str(d["id"]), schemaVersion=int(d.get("schemaVersion", 1)), type=d["type"],
//   target=Target(**d["target"]), params/guards/effects/provenance=dict(d.get(k, {}))
PyObject* ops_from_dicts(PyObject*, PyObject* args) {
  PyObject *items, *op_cls, *tcls;
  Ctor ctor;
  if (!PyArg_ParseTuple(args, "O!O!O!O", &PyList_Type, &items, &PyType_Type, &op_cls, &PyType_Type, &tcls,
                        &ctor.mode_fn))
    return nullptr;
  GcPause gc_pause;
  const Py_ssize_t n = PyList_GET_SIZE(items);
  Ref one(PyLong_FromLong(1));
  if (!one) return nullptr;
  Ref out(PyList_New(n));
  if (!out) return nullptr;
  PyObject* const keys4[4] = {N.params, N.guards, N.effects, N.provenance};
  for (Py_ssize_t k = 0; k < n; ++k) {
    PyObject* d = PyList_GET_ITEM(items, k);
    Ref id_raw(PyObject_GetItem(d, N.id));
    if (!id_raw) return nullptr;
    Ref id(PyObject_Str(id_raw.p));
    if (!id) return nullptr;
    Ref sv_raw(map_get(d, N.schemaVersion, one.p));
    if (!sv_raw) return nullptr;
    Ref sv(PyNumber_Long(sv_raw.p));
    if (!sv) return nullptr;
    Ref ty(PyObject_GetItem(d, N.type));
    if (!ty) return nullptr;
    Ref tg_raw(PyObject_GetItem(d, N.target));
    if (!tg_raw) return nullptr;
    Ref tg;
    {  // Target(**target): the plain-dataclass fast path needs exactly symbolId and addressId
      PyObject *sym = nullptr, *addr = nullptr;
      if (PyDict_CheckExact(tg_raw.p) && PyDict_GET_SIZE(tg_raw.p) == 2) {
        sym = PyDict_GetItemWithError(tg_raw.p, N.symbolId);
        if (!sym && PyErr_Occurred()) return nullptr;
        addr = sym ? PyDict_GetItemWithError(tg_raw.p, N.addressId) : nullptr;
        if (!addr && PyErr_Occurred()) return nullptr;
      }
      const int mode = sym && addr ? ctor.mode((PyTypeObject*)tcls, N.kw_target) : 0;
      if (mode < 0) return nullptr;
      if (mode > 0) {
        PyObject* a[2] = {sym, addr};
        tg.reset(ctor.make((PyTypeObject*)tcls, a, N.kw_target));
      } else {
        Ref kw(PyDict_New());
        if (!kw) return nullptr;
        if (PyDict_Update(kw.p, tg_raw.p) < 0) {  // `**` of a non-mapping: the same TypeError text
          if (PyErr_ExceptionMatches(PyExc_AttributeError)) {
            PyErr_Clear();
            PyErr_Format(PyExc_TypeError, "%.200s() argument after ** must be a mapping, not %.200s",
                         ((PyTypeObject*)tcls)->tp_name, Py_TYPE(tg_raw.p)->tp_name);
          }
          return nullptr;
        }
        tg.reset(PyObject_Call(tcls, N.empty, kw.p));
      }
      if (!tg) return nullptr;
    }
    Ref vals[4];
    for (int q = 0; q < 4; ++q) {  // dict(d.get(k, {}))
      if (PyDict_CheckExact(d)) {
        PyObject* v = PyDict_GetItemWithError(d, keys4[q]);
        if (!v && PyErr_Occurred()) return nullptr;
        vals[q].reset(v ? dict_of(v) : PyDict_New());
      } else {
        Ref dflt(PyDict_New());
        if (!dflt) return nullptr;
        Ref raw(PyObject_CallMethodObjArgs(d, N.get, keys4[q], dflt.p, nullptr));
        if (!raw) return nullptr;
        vals[q].reset(dict_of(raw.p));
      }
      if (!vals[q]) return nullptr;
    }
    PyObject* a8[8] = {id.p, sv.p, ty.p, tg.p, vals[0].p, vals[1].p, vals[2].p, vals[3].p};
    PyObject* op = ctor.make((PyTypeObject*)op_cls, a8, N.kw_op);
    if (!op) return nullptr;
    PyList_SET_ITEM(out.p, k, op);
  }
  return out.release();
}

PyMethodDef methods[] = {
    {"ops_from_dicts", ops_from_dicts, METH_VARARGS, "Op.from_dict over a list (ops.py:89-100)."},
    {"marshal_ops", marshal_ops, METH_VARARGS, "List[Op] -> SoA columns (see marshal.py)."},
    {"materialize_ops", materialize_ops, METH_VARARGS, "device results -> List[Op] (see materialize.py)."},
    {"deep_copy", py_deep_copy, METH_VARARGS, "copy.deepcopy with a native JSON-tree path."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_smx_host", "Native host marshal / materialise.", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__smx_host(void) {
  if (!init_names()) return nullptr;
  return PyModule_Create(&module);
}
