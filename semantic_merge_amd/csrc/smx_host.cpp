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
#include <cstdlib>
#include <cstring>
#include <string>
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

// Whether instances of cls keep the fields `names` as plain instance-dict entries: the
// generic attribute protocol (no __getattribute__ / __getattr__ / __setattr__
// override) and no data descriptor of those names anywhere in the MRO.  Then
// getattr(obj, name) is obj.__dict__[name] when present (else the class attribute),
// and setattr is an instance-dict store.  Decided once per class.
struct PlainFields {
  std::vector<std::pair<PyTypeObject*, bool>> seen;
  bool check(PyTypeObject* cls, PyObject* names) {
    for (auto& e : seen)
      if (e.first == cls) return e.second;
    bool ok = cls->tp_getattro == PyObject_GenericGetAttr && cls->tp_setattro == PyObject_GenericSetAttr &&
              cls->tp_dictoffset != 0;
    for (Py_ssize_t i = 0; ok && i < PyTuple_GET_SIZE(names); ++i) {
      PyObject* d = _PyType_Lookup(cls, PyTuple_GET_ITEM(names, i));  // (borrowed, no error)
      if (d && Py_TYPE(d)->tp_descr_set) ok = false;
    }
    seen.emplace_back(cls, ok);
    return ok;
  }
};

// getattr(obj, name) for a PlainFields class: the instance dict's entry (borrowed) or,
// when it has none, the generic lookup (new reference in *hold).
PyObject* plain_get(PyObject* obj, PyObject* name, Ref& hold) {
  PyObject** dp = _PyObject_GetDictPtr(obj);
  if (dp && *dp && PyDict_CheckExact(*dp)) {
    PyObject* v = PyDict_GetItemWithError(*dp, name);
    if (v || PyErr_Occurred()) return v;
  }
  hold.reset(PyObject_GetAttr(obj, name));
  return hold.p;
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

// lowercase hex digit value, or 0x80 (any other byte)
struct HexTable {
  uint8_t v[256];
  constexpr HexTable() : v() {
    for (int i = 0; i < 256; ++i) v[i] = 0x80;
    for (int i = 0; i < 10; ++i) v['0' + i] = (uint8_t)i;
    for (int i = 0; i < 6; ++i) v['a' + i] = (uint8_t)(10 + i);
  }
};
constexpr HexTable kHex{};

// Canonical lowercase UUID (exact str) -> 128-bit value.  Table-driven and branch-free
// over the 32 digits (a per-character branch chain measured ~0.3 us per id).
bool uuid_key(PyObject* s, uint64_t* hi, uint64_t* lo) {
  if (!PyUnicode_CheckExact(s)) return false;
  if (PyUnicode_READY(s) < 0) {
    PyErr_Clear();
    return false;
  }
  if (PyUnicode_KIND(s) != PyUnicode_1BYTE_KIND || PyUnicode_GET_LENGTH(s) != 36) return false;
  const unsigned char* c = PyUnicode_1BYTE_DATA(s);
  if ((c[8] != '-') | (c[13] != '-') | (c[18] != '-') | (c[23] != '-')) return false;
  // digit positions: 0-7, 9-12, 14-17 (hi); 19-22, 24-35 (lo)
  static constexpr uint8_t pos[32] = {0,  1,  2,  3,  4,  5,  6,  7,  9,  10, 11, 12, 14, 15, 16, 17,
                                      19, 20, 21, 22, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35};
  uint64_t h = 0, l = 0;
  uint8_t bad = 0;
  for (int i = 0; i < 16; ++i) {
    const uint8_t v = kHex.v[c[pos[i]]];
    bad |= v;
    h = (h << 4) | (v & 15u);
  }
  for (int i = 16; i < 32; ++i) {
    const uint8_t v = kHex.v[c[pos[i]]];
    bad |= v;
    l = (l << 4) | (v & 15u);
  }
  if (bad & 0x80) return false;
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

// The int object of id i (borrowed): one per id for the module's lifetime, shared by
// every call (the interners' dict values; no allocation per new value).
PyObject* id_object(long long i) {
  static std::vector<PyObject*> ids;
  if (i < (long long)ids.size()) return ids[(size_t)i];
  if (i >= (1ll << 26)) {  // (beyond 64M ids: no cache, the dict keeps its own reference)
    static Ref last;
    last.reset(PyLong_FromLongLong(i));
    return last.p;
  }
  while ((long long)ids.size() <= i) {
    PyObject* o = PyLong_FromLongLong((long long)ids.size());
    if (!o) return nullptr;
    ids.push_back(o);
  }
  return ids[(size_t)i];
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
    PyObject* v = id_object(id);
    if (!v || PyDict_SetItem(map, key, v) < 0) return -1;
    if (list && PyList_Append(list, key) < 0) return -1;
    return id;
  }
  long long fresh() { return next++; }
};

// ---------------------------------------------------------------- marshal

// One op at a time into growing SoA columns (marshal.py; compose.py:16-18 sort key,
// :64-82 chain values).
struct Marshaler {
  PyObject *kind_rank, *default_ts, *eq_key;
  int unknown, kmove, krename;
  Interner syms, strings, eq;
  std::vector<uint8_t> kind;
  std::vector<uint64_t> ts, hi, lo;
  std::vector<uint32_t> sym;
  std::vector<int32_t> v0, v1;
  Ref ts_list, id_list;
  bool ts_ok = true, all_uuid = true;

  bool init() {
    ts_list.reset(PyList_New(0));
    id_list.reset(PyList_New(0));
    return syms.init(false) && strings.init(true) && eq.init(false) && ts_list && id_list;
  }
  bool sid(PyObject* v, int32_t* dst) {  // strings[str(v)]
    Ref s(PyObject_Str(v));
    if (!s) return false;
    const long long id = strings(s.p);
    if (id < 0) return false;
    *dst = (int32_t)id;
    return true;
  }
  PlainFields plain;  // op / target classes whose fields are read from the instance dict
  // getattr(o, name): the instance dict's entry on a PlainFields class (the same value)
  PyObject* get(PyObject* o, PyObject* name, PyObject* names, Ref& hold) {
    if (plain.check(Py_TYPE(o), names)) return plain_get(o, name, hold);
    hold.reset(PyObject_GetAttr(o, name));
    return hold.p;
  }
  bool add(PyObject* op) {
    const size_t k = kind.size();
    kind.push_back(0);
    ts.push_back(0);
    hi.push_back(0);
    lo.push_back(0);
    sym.push_back(0);
    v0.push_back(-1);
    v1.push_back(-1);
    // precedence.get(op.type, 99) (compose.py:18)
    Ref ht, hp, hi_, hg, hs, hpa;
    PyObject* type = get(op, N.type, N.kw_op, ht);
    if (!type) return false;
    PyObject* r = PyDict_GetItemWithError(kind_rank, type);
    if (!r && PyErr_Occurred()) return false;
    const int kr = r ? (int)PyLong_AsLong(r) : unknown;
    kind[k] = (uint8_t)kr;
    // str(op.provenance.get("timestamp", "1970-01-01T00:00:00Z")) (compose.py:17)
    PyObject* prov = get(op, N.provenance, N.kw_op, hp);
    if (!prov) return false;
    Ref tso(map_get(prov, N.timestamp, default_ts));
    if (!tso) return false;
    Ref tss(PyObject_Str(tso.p));
    if (!tss || PyList_Append(ts_list.p, tss.p) < 0) return false;
    if (ts_ok && !iso_key(tss.p, &ts[k])) ts_ok = false;
    // op.id (compose.py:18)
    PyObject* id = get(op, N.id, N.kw_op, hi_);
    if (!id || PyList_Append(id_list.p, id) < 0) return false;
    if (all_uuid && !uuid_key(id, &hi[k], &lo[k])) all_uuid = false;
    // target.symbolId: dict key / == (compose.py:33,64)
    PyObject* tgt = get(op, N.target, N.kw_op, hg);
    if (!tgt) return false;
    PyObject* s = get(tgt, N.symbolId, N.kw_target, hs);
    if (!s) return false;
    const long long si = syms(s);
    if (si < 0) return false;
    sym[k] = (uint32_t)si;
    if (kr != kmove && kr != krename) return true;
    PyObject* pp = get(op, N.params, N.kw_op, hpa);
    if (!pp) return false;
    Py_INCREF(pp);
    Ref params(pp);
    if (kr == krename) {  // newName: '!=' class (compose.py:66) and str(newName) (compose.py:72)
      Ref name(map_get(params.p, N.newName, Py_None));
      if (!name) return false;
      bool nan = false;
      if (PyFloat_CheckExact(name.p)) {
        nan = std::isnan(PyFloat_AS_DOUBLE(name.p));
      } else if (PyFloat_Check(name.p)) {
        const int ne = PyObject_RichCompareBool(name.p, name.p, Py_NE);
        if (ne < 0) return false;
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
          if (!key) return false;
        }
        const long long c = eq(key.p);
        if (c < 0) return false;
        v0[k] = (int32_t)c;
      }
      return sid(name.p, &v1[k]);
    }
    // moves: str(newAddress), str(newFile or file) (compose.py:75-82)
    Ref addr(map_get(params.p, N.newAddress, Py_None));
    if (!addr) return false;
    if (addr.p != Py_None && !sid(addr.p, &v0[k])) return false;
    Ref nfile(map_get(params.p, N.newFile, Py_None));
    if (!nfile) return false;
    const int truthy = PyObject_IsTrue(nfile.p);
    if (truthy < 0) return false;
    if (!truthy) {
      nfile.reset(map_get(params.p, N.file, Py_None));
      if (!nfile) return false;
    }
    if (nfile.p != Py_None && !sid(nfile.p, &v1[k])) return false;
    return true;
  }
  // (n_sym, strings, ts_ok, id_mode, ts_strs | None, ids | None)
  PyObject* summary() {
    const Py_ssize_t n = (Py_ssize_t)kind.size();
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
};

template <typename T>
bool copy_col(const std::vector<T>& v, PyObject* o, const char* what) {
  Buf b;
  if (!get_buf(o, b, sizeof(T), (Py_ssize_t)v.size(), true, what)) return false;
  if (!v.empty()) std::memcpy(b.v.buf, v.data(), v.size() * sizeof(T));
  return true;
}

bool parse_marshal_args(PyObject* args, PyObject** ops, Marshaler& M, PyObject** cols) {
  return PyArg_ParseTuple(args, "O!O!iiiUOOOOOOOO", &PyList_Type, ops, &PyDict_Type, &M.kind_rank, &M.unknown,
                          &M.kmove, &M.krename, &M.default_ts, &M.eq_key, &cols[0], &cols[1], &cols[2], &cols[3],
                          &cols[4], &cols[5], &cols[6]);
}

bool store_cols(const Marshaler& M, PyObject** cols) {
  return copy_col(M.kind, cols[0], "kind") && copy_col(M.ts, cols[1], "ts") && copy_col(M.hi, cols[2], "oid_hi") &&
         copy_col(M.lo, cols[3], "oid_lo") && copy_col(M.sym, cols[4], "sym") && copy_col(M.v0, cols[5], "v0") &&
         copy_col(M.v1, cols[6], "v1");
}

// marshal_ops(ops, kind_rank, unknown, kmove, krename, default_ts, eq_key,
//             kind, ts, hi, lo, sym, v0, v1)
//   -> (n_sym, strings, ts_ok, id_mode, ts_strs | None, ids | None)
// ts_ok False: ts_strs holds every timestamp string for the rank encoder.
// id_mode 0 UUID, 1 packed, -1: ids holds every id for the Python encoder.
PyObject* marshal_ops(PyObject*, PyObject* args) {
  PyObject* ops;
  PyObject* cols[7];
  Marshaler M;
  if (!parse_marshal_args(args, &ops, M, cols) || !M.init()) return nullptr;
  const Py_ssize_t n = PyList_GET_SIZE(ops);
  M.kind.reserve(n), M.ts.reserve(n), M.hi.reserve(n), M.lo.reserve(n), M.sym.reserve(n), M.v0.reserve(n),
      M.v1.reserve(n);
  for (Py_ssize_t k = 0; k < n; ++k)
    if (!M.add(PyList_GET_ITEM(ops, k))) return nullptr;
  Ref sum(M.summary());  // (packs the short ids into hi / lo)
  if (!sum || !store_cols(M, cols)) return nullptr;
  return sum.release();
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

// *fresh (when given): the copy is a native one -- a tree whose containers nothing else,
// not even the copy itself, refers to -- rather than copy.deepcopy's.
PyObject* deep_copy(PyObject* x, PyObject* deepcopy, bool* fresh = nullptr) {
  if (fresh) *fresh = true;
  if (PyDict_CheckExact(x)) {
    if (PyDict_GET_SIZE(x) == 0) return PyDict_New();
    // a flat dict of atoms (params / provenance as lift.ts writes them): one table copy
    // (copy_tree's first test, without its bookkeeping)
    Py_ssize_t pos = 0;
    PyObject *key, *val;
    bool flat = true;
    while (flat && PyDict_Next(x, &pos, &key, &val)) flat = is_atom(key) && is_atom(val);
    if (flat) return PyDict_Copy(x);
  }
  std::vector<PyObject*> seen;
  bool tree = true;
  PyObject* y = copy_tree(x, seen, &tree, 0);
  if (y || tree) return y;  // copied, or a real error
  if (fresh) *fresh = false;
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
  // mode 1 on a PlainFields class: object.__new__, then the instance dict built at once
  // (what one setattr per field in order leaves: the same keys in the same order)
  PyObject* make_plain(PyTypeObject* cls, PyObject* const* args, PyObject* names) {
    Ref obj(PyBaseObject_Type.tp_new(cls, N.empty, nullptr));
    if (!obj) return nullptr;
    PyObject** dp = _PyObject_GetDictPtr(obj.p);
    if (!dp || *dp) return make_attrs(obj.release(), 1, args, names);
    const Py_ssize_t nf = PyTuple_GET_SIZE(names);
    Ref d(_PyDict_NewPresized(nf));
    if (!d) return nullptr;
    for (Py_ssize_t i = 0; i < nf; ++i)
      if (PyDict_SetItem(d.p, PyTuple_GET_ITEM(names, i), args[i]) < 0) return nullptr;
    *dp = d.release();
    return obj.release();
  }
  PyObject* make_attrs(PyObject* o, int m, PyObject* const* args, PyObject* names) {
    Ref obj(o);
    for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(names); ++i) {
      PyObject* nm = PyTuple_GET_ITEM(names, i);
      const int rc = m == 1 ? PyObject_SetAttr(obj.p, nm, args[i]) : PyObject_GenericSetAttr(obj.p, nm, args[i]);
      if (rc < 0) return nullptr;
    }
    return obj.release();
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

// Software prefetch of the object graph a clone reads, a few ops ahead in output order
// (ops are visited in T order, i.e. in no relation to where they sit in memory: most
// reads were cache misses).  Only reads what earlier stages already pulled in, and
// only objects whose type is checked first; a prefetch never changes behaviour.
inline void pf(const void* p) { __builtin_prefetch(p, 0, 3); }
inline PyObject* inst_dict(PyObject* o) {
  PyObject** dp = _PyObject_GetDictPtr(o);
  return dp ? *dp : nullptr;
}
inline void pf_dict_tables(PyObject* d) {  // the dict's key and value tables
  if (d && PyDict_CheckExact(d)) {
    pf(((PyDictObject*)d)->ma_keys);
    if (((PyDictObject*)d)->ma_values) pf(((PyDictObject*)d)->ma_values);
  }
}
inline void pf_dict_values(PyObject* d) {  // ... and each value object
  if (!d || !PyDict_CheckExact(d)) return;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(d, &pos, &k, &v)) pf(v);
}
struct OpPrefetch {
  PyObject* ops;
  const int32_t* order;
  Py_ssize_t m, n_ops;
  PyObject* at(Py_ssize_t j) const {
    if (j >= m) return nullptr;
    const int32_t s = order[j];
    return s >= 0 && s < n_ops ? PyList_GET_ITEM(ops, s) : nullptr;
  }
  void step(Py_ssize_t t) const {
    if (PyObject* o = at(t + 24)) pf(o);
    if (PyObject* o = at(t + 18)) pf(inst_dict(o));
    if (PyObject* o = at(t + 12)) pf_dict_tables(inst_dict(o));
    if (PyObject* o = at(t + 8)) pf_dict_values(inst_dict(o));  // the field objects
    if (PyObject* o = at(t + 4)) {  // the fields' own tables; the target's dict
      PyObject* d = inst_dict(o);
      if (d && PyDict_CheckExact(d)) {
        Py_ssize_t pos = 0;
        PyObject *k, *v;
        while (PyDict_Next(d, &pos, &k, &v)) {
          if (PyDict_CheckExact(v)) pf_dict_tables(v);
          else if (!PyUnicode_CheckExact(v) && !PyLong_CheckExact(v)) pf(inst_dict(v));
        }
      }
    }
    if (PyObject* o = at(t + 2)) {  // the fields' values; the target's tables
      PyObject* d = inst_dict(o);
      if (d && PyDict_CheckExact(d)) {
        Py_ssize_t pos = 0;
        PyObject *k, *v;
        while (PyDict_Next(d, &pos, &k, &v)) {
          if (PyDict_CheckExact(v)) pf_dict_values(v);
          else if (!PyUnicode_CheckExact(v) && !PyLong_CheckExact(v)) pf_dict_tables(inst_dict(v));
        }
      }
    }
  }
};


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
  PlainFields plain;
  const OpPrefetch pfo{ops, order, m, n_ops};
  for (Py_ssize_t t = 0; t < m; ++t) {
    pfo.step(t);
    const int32_t src = order[t];
    if (src < 0 || src >= n_ops) {
      PyErr_SetString(PyExc_IndexError, "source index out of range");
      return nullptr;
    }
    PyObject* op = PyList_GET_ITEM(ops, src);
    // Fast path: a plain (non-frozen) dataclass Op over a plain dataclass Target, both
    // with instance-dict fields (PlainFields).  The clone is then built already
    // materialised -- the final target, the edited params -- which is what constructing
    // it and then assigning its attributes (compose.py:30-49 on :117-127) leaves behind:
    // the generated __init__ only stores its arguments.
    {
      PyTypeObject* ocls = Py_TYPE(op);
      const int om = ctor.mode(ocls, N.kw_op);
      if (om < 0) return nullptr;
      if (om == 1 && plain.check(ocls, N.kw_op)) {
        Ref h0, h1, h2, h3, h4, h5, h6, h7, h8, h9;
        PyObject* tg = plain_get(op, N.target, h0);
        if (!tg) return nullptr;
        PyTypeObject* tcls = Py_TYPE(tg);
        const int tm = ctor.mode(tcls, N.kw_target);
        if (tm < 0) return nullptr;
        if (tm >= 1 && plain.check(tcls, N.kw_target)) {
          PyObject *id, *sv, *ty, *tsym, *taddr;
          if (!(id = plain_get(op, N.id, h1)) || !(sv = plain_get(op, N.schemaVersion, h2)) ||
              !(ty = plain_get(op, N.type, h3)) || !(tsym = plain_get(tg, N.symbolId, h4)) ||
              !(taddr = plain_get(tg, N.addressId, h5)))
            return nullptr;
          const int k = kind[src];
          const int32_t a = addr[t], f = file[t], c = ctx[t];
          PyObject *sa = nullptr, *sf = nullptr, *sc = nullptr;
          if ((a >= 0 && !(sa = str_at(a))) || (f >= 0 && !(sf = str_at(f))) || (c >= 0 && !(sc = str_at(c))))
            return nullptr;
          PyObject* ta[2] = {tsym, sa ? sa : taddr};
          bool p_fresh = false;
          Ref p, g, e, pr, ntgt(tm == 1 ? ctor.make_plain(tcls, ta, N.kw_target) : ctor.make(tcls, ta, N.kw_target));
          if (!ntgt) return nullptr;
          {
            PyObject* x;
            if (!(x = plain_get(op, N.params, h6)) || !(p.reset(deep_copy(x, deepcopy, &p_fresh)), p)) return nullptr;
            if (!(x = plain_get(op, N.guards, h7)) || !(g.reset(deep_copy(x, deepcopy)), g)) return nullptr;
            if (!(x = plain_get(op, N.effects, h8)) || !(e.reset(deep_copy(x, deepcopy)), e)) return nullptr;
            if (!(x = plain_get(op, N.provenance, h9)) || !(pr.reset(deep_copy(x, deepcopy)), pr)) return nullptr;
          }
          if (k == kmove) {
            if (sa && PyObject_SetItem(p.p, N.newAddress, sa) < 0) return nullptr;
            if (sf && PyObject_SetItem(p.p, N.newFile, sf) < 0) return nullptr;
          }
          if (k == krename && sf &&
              (PyObject_SetItem(p.p, N.newFile, sf) < 0 || PyObject_SetItem(p.p, N.file, sf) < 0))
            return nullptr;
          if (sc && k != krename) {  // {**params, "renameContext": ...}: a fresh dict
            if (p_fresh && PyDict_CheckExact(p.p)) {  // (a native copy: referred to from nowhere else)
              if (PyDict_SetItem(p.p, N.renameContext, sc) < 0) return nullptr;
            } else {
              Ref nd(PyDict_New());
              if (!nd || PyDict_Update(nd.p, p.p) < 0 || PyDict_SetItem(nd.p, N.renameContext, sc) < 0)
                return nullptr;
              p.reset(nd.release());
            }
          }
          PyObject* a8[8] = {id, sv, ty, ntgt.p, p.p, g.p, e.p, pr.p};
          PyObject* clone = ctor.make_plain(ocls, a8, N.kw_op);
          if (!clone) return nullptr;
          PyList_SET_ITEM(out.p, t, clone);
          continue;
        }
      }
    }
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

// Op.from_dict(d) (ops.py:89-100) in the same evaluation order and with the same
// coercions (new reference):
//   id=str(d["id"]), schemaVersion=int(d.get("schemaVersion", 1)), type=d["type"],
//   target=Target(**d["target"]), params/guards/effects/provenance=dict(d.get(k, {}))
PyObject* op_from_dict(PyObject* d, Ctor& ctor, PyObject* op_cls, PyObject* tcls, PyObject* one) {
  PyObject* const k4[4] = {N.params, N.guards, N.effects, N.provenance};
  Ref id_raw(PyObject_GetItem(d, N.id));
  if (!id_raw) return nullptr;
  Ref id(PyObject_Str(id_raw.p));
  if (!id) return nullptr;
  Ref sv_raw(map_get(d, N.schemaVersion, one));
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
      PyObject* v = PyDict_GetItemWithError(d, k4[q]);
      if (!v && PyErr_Occurred()) return nullptr;
      vals[q].reset(v ? dict_of(v) : PyDict_New());
    } else {
      Ref dflt(PyDict_New());
      if (!dflt) return nullptr;
      Ref raw(PyObject_CallMethodObjArgs(d, N.get, k4[q], dflt.p, nullptr));
      if (!raw) return nullptr;
      vals[q].reset(dict_of(raw.p));
    }
    if (!vals[q]) return nullptr;
  }
  PyObject* a8[8] = {id.p, sv.p, ty.p, tg.p, vals[0].p, vals[1].p, vals[2].p, vals[3].p};
  return ctor.make((PyTypeObject*)op_cls, a8, N.kw_op);
}

// ops_from_dicts(items, op_cls, target_cls, ctor_mode) -> List[Op]: Op.from_dict of every item.
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
  for (Py_ssize_t k = 0; k < n; ++k) {
    PyObject* op = op_from_dict(PyList_GET_ITEM(items, k), ctor, op_cls, tcls, one.p);
    if (!op) return nullptr;
    PyList_SET_ITEM(out.p, k, op);
  }
  return out.release();
}

// ---------------------------------------------------------------- JSON (ops.py:112-118)

// json.JSONDecodeError(msg, doc, pos) -- what orjson.loads raises (orjson.JSONDecodeError
// subclasses it, and ValueError).  pos counts characters, as the json module's do.
void raise_json_error(const char* what, const char* b, const char* e, const char* at) {
  Ref js(PyImport_ImportModule("json"));
  Ref cls(js ? PyObject_GetAttrString(js.p, "JSONDecodeError") : nullptr);
  Ref doc(PyUnicode_DecodeUTF8(b, e - b, "replace"));
  Ref pre(PyUnicode_DecodeUTF8(b, at - b, "replace"));
  if (!cls || !doc || !pre) return;
  Ref exc(PyObject_CallFunction(cls.p, "sOn", what, doc.p, PyUnicode_GET_LENGTH(pre.p)));
  if (exc) PyErr_SetObject(cls.p, exc.p);
}

// A strict JSON reader with the standard json module's results (dict / list / str /
// int / float / True / False / None; duplicate keys: the last wins; big integers
// exact; float(token) for the rest) and orjson's input rules: NaN / Infinity and lone
// surrogate escapes rejected, no control characters inside strings, nesting up to 1024,
// nothing after the value; errors are json.JSONDecodeError.
struct JsonReader {
  const char* p;
  const char* b;
  const char* e;
  PyObject* memo;  // key strings seen so far (json's memo)
  int depth = 0;
  // raw key text (no escapes, <= 32 bytes) -> its str: one object per distinct key
  // without building a str per occurrence
  struct KeySlot {
    const char* s = nullptr;
    int n = 0;
    PyObject* k = nullptr;  // borrowed from memo
  };
  KeySlot keys[256];

  PyObject* key() {  // p at the opening quote; new reference
    const char* s0 = p + 1;
    const char* q = s0;
    while (q < e && q - s0 <= 32 && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
    if (q < e && *q == '"' && q - s0 <= 32) {
      const int n = (int)(q - s0);
      uint32_t h = 2166136261u;
      for (int i = 0; i < n; ++i) h = (h ^ (unsigned char)s0[i]) * 16777619u;
      for (int probe = 0; probe < 8; ++probe) {
        KeySlot& ks = keys[(h + probe) & 255];
        if (ks.k && ks.n == n && std::memcmp(ks.s, s0, (size_t)n) == 0) {
          p = q + 1;
          Py_INCREF(ks.k);
          return ks.k;
        }
        if (!ks.k) {
          Ref k(string());
          if (!k) return nullptr;
          PyObject* m = PyDict_SetDefault(memo, k.p, k.p);
          if (!m) return nullptr;
          ks.s = s0;
          ks.n = n;
          ks.k = m;
          Py_INCREF(m);
          return m;
        }
      }
    }
    Ref k(string());
    if (!k) return nullptr;
    PyObject* m = PyDict_SetDefault(memo, k.p, k.p);  // one object per key text
    if (!m) return nullptr;
    Py_INCREF(m);
    return m;
  }

  bool fail(const char* what) {
    if (!PyErr_Occurred()) raise_json_error(what, b, e, p < e ? p : e);
    return false;
  }
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static int hex4(const char* q) {
    int v = 0;
    for (int i = 0; i < 4; ++i) {
      const int h = hexval((unsigned char)(q[i] | ((q[i] >= 'A' && q[i] <= 'F') ? 0x20 : 0)));
      if (h < 0) return -1;
      v = v << 4 | h;
    }
    return v;
  }
  PyObject* string() {  // p at the opening quote
    ++p;
    const char* s0 = p;
    bool esc = false;
    while (p < e && *p != '"') {
      const unsigned char c = (unsigned char)*p;
      if (c < 0x20) return fail("control character in string"), nullptr;
      if (c == '\\') {
        esc = true;
        if (++p >= e) break;
      }
      ++p;
    }
    if (p >= e) return fail("unterminated string"), nullptr;
    const char* s1 = p++;
    if (!esc) {
      PyObject* r = PyUnicode_DecodeUTF8(s0, s1 - s0, "strict");
      if (!r && PyErr_ExceptionMatches(PyExc_UnicodeDecodeError)) PyErr_Clear(), p = s0, fail("invalid UTF-8");
      return r;
    }
    std::vector<Py_UCS4> u;
    u.reserve((size_t)(s1 - s0));
    for (const char* q = s0; q < s1;) {
      const unsigned char c = (unsigned char)*q;
      if (c == '\\') {
        const char x = q[1];
        q += 2;
        switch (x) {
          case '"': u.push_back('"'); break;
          case '\\': u.push_back('\\'); break;
          case '/': u.push_back('/'); break;
          case 'b': u.push_back('\b'); break;
          case 'f': u.push_back('\f'); break;
          case 'n': u.push_back('\n'); break;
          case 'r': u.push_back('\r'); break;
          case 't': u.push_back('\t'); break;
          case 'u': {
            if (s1 - q < 4) return p = q, fail("truncated \\u escape"), nullptr;
            int cp = hex4(q);
            if (cp < 0) return p = q, fail("invalid \\u escape"), nullptr;
            q += 4;
            if (cp >= 0xD800 && cp <= 0xDBFF && s1 - q >= 6 && q[0] == '\\' && q[1] == 'u') {
              const int lo2 = hex4(q + 2);  // a surrogate pair
              if (lo2 >= 0xDC00 && lo2 <= 0xDFFF) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo2 - 0xDC00);
                q += 6;
              }
            }
            // a lone surrogate is not UTF-8: orjson rejects it (the json module keeps it)
            if (cp >= 0xD800 && cp <= 0xDFFF) return p = q - 6, fail("lone surrogate in \\u escape"), nullptr;
            u.push_back((Py_UCS4)cp);
            break;
          }
          default:
            return p = q - 1, fail("invalid escape"), nullptr;
        }
        continue;
      }
      // one UTF-8 sequence (validated by the decoder)
      int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
      if (!len || q + len > s1) return p = q, fail("invalid UTF-8"), nullptr;
      Ref one_cp(PyUnicode_DecodeUTF8(q, len, "strict"));
      if (!one_cp) {
        if (PyErr_ExceptionMatches(PyExc_UnicodeDecodeError)) PyErr_Clear(), p = q, fail("invalid UTF-8");
        return nullptr;
      }
      u.push_back(PyUnicode_READ_CHAR(one_cp.p, 0));
      q += len;
    }
    return PyUnicode_FromKindAndData(PyUnicode_4BYTE_KIND, u.data(), (Py_ssize_t)u.size());
  }
  PyObject* number() {
    const char* s0 = p;
    bool isf = false;
    if (p < e && *p == '-') ++p;
    if (p < e && *p == '0') {
      ++p;
    } else if (p < e && *p >= '1' && *p <= '9') {
      while (p < e && *p >= '0' && *p <= '9') ++p;
    } else {
      return fail("invalid number"), nullptr;
    }
    if (p < e && *p == '.') {
      isf = true;
      ++p;
      if (!(p < e && *p >= '0' && *p <= '9')) return fail("invalid number"), nullptr;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      isf = true;
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (!(p < e && *p >= '0' && *p <= '9')) return fail("invalid number"), nullptr;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    const size_t len = (size_t)(p - s0);
    if (!isf && len <= 18) {  // fits int64: digits straight from the text
      long long v = 0;
      const char* q = s0 + (*s0 == '-');
      for (; q < p; ++q) v = v * 10 + (*q - '0');
      return PyLong_FromLongLong(*s0 == '-' ? -v : v);
    }
    std::string tok(s0, len);
    if (isf) {
      const double v = PyOS_string_to_double(tok.c_str(), nullptr, nullptr);
      if (v == -1.0 && PyErr_Occurred()) return nullptr;
      return PyFloat_FromDouble(v);
    }
    return PyLong_FromString(tok.c_str(), nullptr, 10);
  }
  bool lit(const char* w) {
    const size_t n = std::strlen(w);
    if ((size_t)(e - p) >= n && std::memcmp(p, w, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  PyObject* value() {
    ws();
    if (p >= e) return fail("unexpected end"), nullptr;
    switch (*p) {
      case '{': {
        if (++depth > 1024) return fail("nesting too deep"), nullptr;
        ++p;
        Ref d(PyDict_New());
        if (!d) return nullptr;
        ws();
        if (p < e && *p == '}') {
          ++p;
          --depth;
          return d.release();
        }
        for (;;) {
          ws();
          if (p >= e || *p != '"') return fail("expected a key"), nullptr;
          Ref k(key());
          if (!k) return nullptr;
          ws();
          if (p >= e || *p != ':') return fail("expected ':'"), nullptr;
          ++p;
          Ref v(value());
          if (!v || PyDict_SetItem(d.p, k.p, v.p) < 0) return nullptr;
          ws();
          if (p < e && *p == ',') {
            ++p;
            continue;
          }
          if (p < e && *p == '}') {
            ++p;
            break;
          }
          return fail("expected ',' or '}'"), nullptr;
        }
        --depth;
        return d.release();
      }
      case '[': {
        if (++depth > 1024) return fail("nesting too deep"), nullptr;
        ++p;
        Ref l(PyList_New(0));
        if (!l) return nullptr;
        ws();
        if (p < e && *p == ']') {
          ++p;
          --depth;
          return l.release();
        }
        for (;;) {
          Ref v(value());
          if (!v || PyList_Append(l.p, v.p) < 0) return nullptr;
          ws();
          if (p < e && *p == ',') {
            ++p;
            continue;
          }
          if (p < e && *p == ']') {
            ++p;
            break;
          }
          return fail("expected ',' or ']'"), nullptr;
        }
        --depth;
        return l.release();
      }
      case '"':
        return string();
      case 't':
        if (lit("true")) Py_RETURN_TRUE;
        break;
      case 'f':
        if (lit("false")) Py_RETURN_FALSE;
        break;
      case 'n':
        if (lit("null")) Py_RETURN_NONE;
        break;
      case 'N':
      case 'I':
        return fail("NaN / Infinity are not JSON"), nullptr;
      default:
        if (*p == '-' && p + 1 < e && p[1] == 'I') return fail("NaN / Infinity are not JSON"), nullptr;
        if (*p == '-' || (*p >= '0' && *p <= '9')) return number();
    }
    return fail("unexpected character"), nullptr;
  }
  PyObject* document() {
    Ref v(value());
    if (!v) return nullptr;
    ws();
    if (p != e) return fail("extra data"), nullptr;
    return v.release();
  }
};

// UTF-8 view of a str / bytes-like argument (bytes are taken as UTF-8).
bool utf8_of(PyObject* x, Ref& hold, const char** s, Py_ssize_t* n) {
  if (PyUnicode_Check(x)) {
    *s = PyUnicode_AsUTF8AndSize(x, n);
    if (!*s && PyErr_ExceptionMatches(PyExc_UnicodeEncodeError)) {  // lone surrogates: orjson's error
      PyErr_Clear();
      Ref js(PyImport_ImportModule("json"));
      Ref cls(js ? PyObject_GetAttrString(js.p, "JSONDecodeError") : nullptr);
      if (cls) {
        Ref exc(PyObject_CallFunction(cls.p, "sOn", "str is not valid UTF-8: surrogates not allowed", x,
                                      (Py_ssize_t)0));
        if (exc) PyErr_SetObject(cls.p, exc.p);
      }
    }
    return *s != nullptr;
  }
  hold.reset(PyBytes_FromObject(x));
  if (!hold) return false;
  *s = PyBytes_AS_STRING(hold.p);
  *n = PyBytes_GET_SIZE(hold.p);
  return true;
}

PyObject* json_loads(PyObject*, PyObject* x) {
  GcPause gc_pause;
  Ref hold, memo(PyDict_New());
  const char* s;
  Py_ssize_t n;
  if (!memo || !utf8_of(x, hold, &s, &n)) return nullptr;
  JsonReader R{s, s, s + n, memo.p};
  return R.document();
}

// decode_oplogs(texts, op_cls, target_cls, ctor_mode, kind_rank, unknown, kmove, krename,
//               default_ts, eq_key)
//   -> (per-text op lists, marshal summary (as marshal_ops), kind, ts, hi, lo, sym, v0, v1)
// OpLog.from_json of each text (ops.py:116-118) and the compose SoA of all of them
// together (marshal_ops over the concatenation) in one pass: each parsed op object
// is built and marshalled before the next is read.
PyObject* decode_oplogs(PyObject*, PyObject* args) {
  PyObject *texts, *op_cls, *tcls;
  Ctor ctor;
  Marshaler M;
  if (!PyArg_ParseTuple(args, "O!O!O!OO!iiiUO", &PyTuple_Type, &texts, &PyType_Type, &op_cls, &PyType_Type, &tcls,
                        &ctor.mode_fn, &PyDict_Type, &M.kind_rank, &M.unknown, &M.kmove, &M.krename,
                        &M.default_ts, &M.eq_key) ||
      !M.init())
    return nullptr;
  GcPause gc_pause;
  Ref one(PyLong_FromLong(1)), lists(PyTuple_New(PyTuple_GET_SIZE(texts)));
  if (!one || !lists) return nullptr;
  // The reference decodes each text whole (orjson.loads), then builds its ops
  // (Op.from_dict per item, ops.py:116-118), and compose marshals after both: a JSON
  // error anywhere in a text comes before an item error of that text, which comes
  // before any marshalling error.  Items are built while the text is read; the first
  // item / marshalling error is held back until its turn.
  struct Held {
    PyObject *t = nullptr, *v = nullptr, *tb = nullptr;
    bool set() const { return t != nullptr; }
    void take() { PyErr_Fetch(&t, &v, &tb); }
    PyObject* raise() {
      PyErr_Restore(t, v, tb);
      t = v = tb = nullptr;
      return nullptr;
    }
    ~Held() {
      Py_XDECREF(t);
      Py_XDECREF(v);
      Py_XDECREF(tb);
    }
  } marshal_err;
  for (Py_ssize_t t = 0; t < PyTuple_GET_SIZE(texts); ++t) {
    Held item_err;
    auto add_item = [&](PyObject* item, PyObject* out) -> bool {  // false: a real failure
      if (item_err.set()) return true;  // the reference stopped at the first failing item
      Ref op(op_from_dict(item, ctor, op_cls, tcls, one.p));
      if (!op) {
        item_err.take();
        return true;
      }
      if (PyList_Append(out, op.p) < 0) return false;
      if (!marshal_err.set() && !M.add(op.p)) marshal_err.take();
      return true;
    };
    Ref hold, memo(PyDict_New());
    const char* s;
    Py_ssize_t n;
    if (!memo || !utf8_of(PyTuple_GET_ITEM(texts, t), hold, &s, &n)) return nullptr;
    JsonReader R{s, s, s + n, memo.p};
    Ref out(PyList_New(0));
    if (!out) return nullptr;
    R.ws();
    if (R.p < R.e && *R.p == '[') {  // the usual document: ops decoded as they are read
      ++R.p;
      R.depth = 1;  // the outer array counts toward the nesting limit
      R.ws();
      bool first = true;
      while (!(R.p < R.e && *R.p == ']')) {
        if (!first) {
          if (!(R.p < R.e && *R.p == ',')) return R.fail("expected ',' or ']'"), nullptr;
          ++R.p;
        }
        first = false;
        Ref item(R.value());
        if (!item) return nullptr;
        if (!add_item(item.p, out.p)) return nullptr;
        R.ws();
      }
      ++R.p;
      R.ws();
      if (R.p != R.e) return R.fail("extra data"), nullptr;
    } else {  // any other document: iterate it as the reference's list comprehension does
      Ref doc(R.document());
      if (!doc) return nullptr;
      Ref it(PyObject_GetIter(doc.p));
      if (!it) return nullptr;
      while (PyObject* raw = PyIter_Next(it.p)) {
        Ref item(raw);
        if (!add_item(item.p, out.p)) return nullptr;
      }
      if (PyErr_Occurred()) return nullptr;
    }
    if (item_err.set()) return item_err.raise();
    PyTuple_SET_ITEM(lists.p, t, out.release());
  }
  if (marshal_err.set()) return marshal_err.raise();
  Ref sum(M.summary());
  if (!sum) return nullptr;
  auto col = [](const void* d, size_t bytes) { return PyByteArray_FromStringAndSize((const char*)d, (Py_ssize_t)bytes); };
  return Py_BuildValue("OONNNNNNN", lists.p, sum.p, col(M.kind.data(), M.kind.size()),
                       col(M.ts.data(), M.ts.size() * 8), col(M.hi.data(), M.hi.size() * 8),
                       col(M.lo.data(), M.lo.size() * 8), col(M.sym.data(), M.sym.size() * 4),
                       col(M.v0.data(), M.v0.size() * 4), col(M.v1.data(), M.v1.size() * 4));
}

PyMethodDef methods[] = {
    {"ops_from_dicts", ops_from_dicts, METH_VARARGS, "Op.from_dict over a list (ops.py:89-100)."},
    {"marshal_ops", marshal_ops, METH_VARARGS, "List[Op] -> SoA columns (see marshal.py)."},
    {"materialize_ops", materialize_ops, METH_VARARGS, "device results -> List[Op] (see materialize.py)."},
    {"deep_copy", py_deep_copy, METH_VARARGS, "copy.deepcopy with a native JSON-tree path."},
    {"json_loads", json_loads, METH_O, "strict JSON -> Python objects (orjson's input rules)."},
    {"decode_oplogs", decode_oplogs, METH_VARARGS, "OpLog.from_json of each text + their compose SoA."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_smx_host", "Native host marshal / materialise.", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__smx_host(void) {
  if (!init_names()) return nullptr;
  return PyModule_Create(&module);
}
