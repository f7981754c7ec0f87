// CPython front-end of the native host compiler: flattens the caller's
// hash-consed smt.node DAG straight from the Python objects (one walk, no
// per-node Python code) into an mgc_input and runs mgc_compile
// (include/mythcc.h).  Built with mg_compile.cpp into the extension module
// mythril_amd/lib/_mythcc*.so; mythril_amd/ccompile.py wraps it.
//
// _mythcc.compile(constraints, probes, ops, tables, default_entries, nreg,
//                 extra, leaf_pools, const_keys, solve, remat_mode, remat_k,
//                 keep_clean, search_hints, abi_presets)
//   -> (rc, error, code bytes, table bytes, n_const_values, meta json)
// `ops` maps operator names to mgc_source_ops() codes, `tables` is a list of
// (name, size), `extra` the extra constants as 32-byte little-endian rows.

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "mythcc.h"

#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

PyObject *s_op, *s_sort, *s_width, *s_dom, *s_args, *s_params, *s_id, *s_enc;

struct Flat {
    std::vector<int32_t> op, sort, width, dom, arg_off{0}, args, str, cval_off;
    std::vector<int64_t> id, p0, p1;
    std::vector<uint32_t> cval;
    std::string strings;
    int32_t n_strings = 0;
    std::unordered_map<std::string, int32_t> sidx;
    std::unordered_map<PyObject*, int32_t> index;

    int32_t intern(const char* s, Py_ssize_t n) {
        std::string k(s, (size_t)n);
        auto it = sidx.find(k);
        if (it != sidx.end()) return it->second;
        strings.append(k);
        strings.push_back('\0');
        sidx.emplace(std::move(k), n_strings);
        return n_strings++;
    }
};

// attribute as a new reference, or nullptr with an exception set
inline PyObject* attr(PyObject* o, PyObject* name) { return PyObject_GetAttr(o, name); }

bool as_long(PyObject* o, PyObject* name, long long& out) {
    PyObject* v = attr(o, name);
    if (!v) return false;
    out = v == Py_None ? 0 : PyLong_AsLongLong(v);
    Py_DECREF(v);
    return !PyErr_Occurred();
}

bool str_of(PyObject* v, Flat& f, int32_t& out) {
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(v, &n);
    if (!s) return false;
    out = f.intern(s, n);
    return true;
}

// A node's own fields as the walk needs them, computed once per node and
// cached on it (Node._enc): (op code, sort code, width, dom, id, p0, p1,
// name or None, numeral limbs as bytes or None).  Nodes are immutable and
// hash-consed, so a LASER stream's later queries, which share most of their
// DAG with earlier ones, read one tuple per node instead of seven attributes.
PyObject* encode(PyObject* node, PyObject* ops, int other) {
    PyObject* op = attr(node, s_op);
    if (!op) return nullptr;
    PyObject* code = PyDict_GetItemWithError(ops, op);         // borrowed
    int c = code ? (int)PyLong_AsLong(code) : other;
    if (PyErr_Occurred()) { Py_DECREF(op); return nullptr; }
    Py_ssize_t oplen;
    const char* opname = PyUnicode_AsUTF8AndSize(op, &oplen);
    if (!opname) { Py_DECREF(op); return nullptr; }
    std::string name(opname, (size_t)oplen);

    PyObject* sort = attr(node, s_sort);
    if (!sort) { Py_DECREF(op); return nullptr; }
    int sc;
    if (PyUnicode_CompareWithASCIIString(sort, "bv") == 0) sc = MGC_SORT_BV;
    else if (PyUnicode_CompareWithASCIIString(sort, "bool") == 0) sc = MGC_SORT_BOOL;
    else sc = MGC_SORT_ARRAY;
    Py_DECREF(sort);
    long long width, dom, id;
    if (!as_long(node, s_width, width) || !as_long(node, s_dom, dom) || !as_long(node, s_id, id)) {
        Py_DECREF(op);
        return nullptr;
    }
    PyObject* params = attr(node, s_params);
    if (!params) { Py_DECREF(op); return nullptr; }
    PyObject* ps = PySequence_Fast(params, "params");
    Py_DECREF(params);
    if (!ps) { Py_DECREF(op); return nullptr; }
    Py_ssize_t np_ = PySequence_Fast_GET_SIZE(ps);
    PyObject** pv = PySequence_Fast_ITEMS(ps);
    long long p0 = 0, p1 = 0;
    PyObject* str = Py_None;
    PyObject* cval = Py_None;
    Py_INCREF(Py_None);
    Py_INCREF(Py_None);
    bool ok = true;
    if (name == "bvnum" && np_ >= 1) {
        size_t nl = (size_t)(width + 31) / 32;
        std::vector<unsigned char> buf(4 * nl, 0);
        ok = _PyLong_AsByteArray((PyLongObject*)pv[0], buf.data(), buf.size(), 1, 0) == 0;
        if (ok) {
            Py_DECREF(cval);
            cval = PyBytes_FromStringAndSize((const char*)buf.data(), (Py_ssize_t)buf.size());
            ok = cval != nullptr;
        }
    } else if ((name == "var" || name == "array") && np_ >= 1) {
        Py_DECREF(str); str = pv[0]; Py_INCREF(str);
    } else if (name == "apply" && np_ >= 2) {
        Py_DECREF(str); str = pv[0]; Py_INCREF(str);
        p0 = PyLong_AsLongLong(pv[1]);
        ok = !PyErr_Occurred();
    } else if (name == "extract" && np_ >= 2) {
        p0 = PyLong_AsLongLong(pv[0]);
        p1 = PyLong_AsLongLong(pv[1]);
        ok = !PyErr_Occurred();
    } else if ((name == "zero_extend" || name == "sign_extend") && np_ >= 1) {
        p0 = PyLong_AsLongLong(pv[0]);
        ok = !PyErr_Occurred();
    } else if (c == other) {
        Py_DECREF(str); str = op; Py_INCREF(str);
    }
    Py_DECREF(ps);
    Py_DECREF(op);
    if (!ok) { Py_XDECREF(str); Py_XDECREF(cval); return nullptr; }
    PyObject* t = Py_BuildValue("(iiLLLLLNN)", c, sc, width, dom, id, p0, p1, str, cval);
    if (t && PyObject_SetAttr(node, s_enc, t) < 0) PyErr_Clear();   // a node without the slot
    return t;
}

// one node's own fields (operands already indexed; `seq` its args as a fast
// sequence)
bool add_node(PyObject* node, PyObject* seq, PyObject* ops, int other, Flat& f) {
    PyObject* t = PyObject_GetAttr(node, s_enc);
    if (!t) {
        PyErr_Clear();
        t = encode(node, ops, other);
        if (!t) return false;
    }
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 9) {
        Py_DECREF(t);
        PyErr_SetString(PyExc_TypeError, "Node._enc is not a walk record");
        return false;
    }
    const int c = (int)PyLong_AsLong(PyTuple_GET_ITEM(t, 0));
    const int sc = (int)PyLong_AsLong(PyTuple_GET_ITEM(t, 1));
    const long long width = PyLong_AsLongLong(PyTuple_GET_ITEM(t, 2));
    const long long dom = PyLong_AsLongLong(PyTuple_GET_ITEM(t, 3));
    const long long id = PyLong_AsLongLong(PyTuple_GET_ITEM(t, 4));
    const long long p0 = PyLong_AsLongLong(PyTuple_GET_ITEM(t, 5));
    const long long p1 = PyLong_AsLongLong(PyTuple_GET_ITEM(t, 6));
    PyObject* so = PyTuple_GET_ITEM(t, 7);
    PyObject* co = PyTuple_GET_ITEM(t, 8);
    if (PyErr_Occurred()) { Py_DECREF(t); return false; }
    Py_ssize_t na = PySequence_Fast_GET_SIZE(seq);
    for (Py_ssize_t i = 0; i < na; i++) {
        auto it = f.index.find(PySequence_Fast_GET_ITEM(seq, i));
        if (it == f.index.end()) {
            Py_DECREF(t);
            PyErr_SetString(PyExc_RuntimeError, "operand visited after its user");
            return false;
        }
        f.args.push_back(it->second);
    }
    int32_t str = -1, cv = -1;
    if (so != Py_None && !str_of(so, f, str)) { Py_DECREF(t); return false; }
    if (co != Py_None) {
        const Py_ssize_t nb = PyBytes_GET_SIZE(co);
        cv = (int32_t)f.cval.size();
        f.cval.resize(f.cval.size() + (size_t)nb / 4, 0);
        std::memcpy(f.cval.data() + cv, PyBytes_AS_STRING(co), (size_t)nb);
    }
    Py_DECREF(t);
    f.op.push_back(c);
    f.sort.push_back(sc);
    f.width.push_back((int32_t)width);
    f.dom.push_back((int32_t)dom);
    f.id.push_back(id);
    f.arg_off.push_back((int32_t)f.args.size());
    f.p0.push_back(p0);
    f.p1.push_back(p1);
    f.str.push_back(str);
    f.cval_off.push_back(cv);
    f.index.emplace(node, (int32_t)(f.op.size() - 1));
    return true;
}

// post-order walk (operands first) from every root not yet indexed
bool walk(PyObject* root, PyObject* ops, int other, Flat& f) {
    if (f.index.count(root)) return true;
    struct It { PyObject* node; PyObject* seq; Py_ssize_t next; };
    std::vector<It> stack;
    auto push = [&](PyObject* n) -> bool {
        PyObject* args = attr(n, s_args);
        if (!args) return false;
        PyObject* seq = PySequence_Fast(args, "args");
        Py_DECREF(args);
        if (!seq) return false;
        stack.push_back({n, seq, 0});
        return true;
    };
    if (!push(root)) return false;
    std::unordered_map<PyObject*, char> open;
    open[root] = 1;
    while (!stack.empty()) {
        It& it = stack.back();
        if (it.next < PySequence_Fast_GET_SIZE(it.seq)) {
            PyObject* a = PySequence_Fast_GET_ITEM(it.seq, it.next++);
            if (f.index.count(a) || open.count(a)) continue;
            open[a] = 1;
            if (!push(a)) goto fail;
            continue;
        }
        {
            PyObject* n = it.node;
            PyObject* seq = it.seq;
            stack.pop_back();
            const bool ok = add_node(n, seq, ops, other, f);
            Py_DECREF(seq);
            if (!ok) goto fail;
        }
    }
    return true;
fail:
    for (auto& it : stack) Py_DECREF(it.seq);
    return false;
}

PyObject* py_compile(PyObject*, PyObject* a) {
    PyObject *cons, *probes, *ops, *tables, *extra;
    int default_entries, nreg, leaf_pools, const_keys, solve, remat_mode, remat_k, keep_clean;
    int search_hints, abi_presets;
    if (!PyArg_ParseTuple(a, "OOO!OiiSiiiiiiii", &cons, &probes, &PyDict_Type, &ops, &tables,
                          &default_entries, &nreg, &extra, &leaf_pools, &const_keys, &solve,
                          &remat_mode, &remat_k, &keep_clean, &search_hints, &abi_presets))
        return nullptr;
    PyObject* oth = PyDict_GetItemString(ops, "?");
    if (!oth) { PyErr_SetString(PyExc_KeyError, "ops has no '?'"); return nullptr; }
    int other = (int)PyLong_AsLong(oth);
    Flat f;
    std::vector<int32_t> ci, pi;
    for (PyObject* lst : {cons, probes}) {
        PyObject* seq = PySequence_Fast(lst, "constraints / probes");
        if (!seq) return nullptr;
        Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
        for (Py_ssize_t i = 0; i < n; i++)
            if (!walk(PySequence_Fast_GET_ITEM(seq, i), ops, other, f)) { Py_DECREF(seq); return nullptr; }
        for (Py_ssize_t i = 0; i < n; i++)
            (lst == cons ? ci : pi).push_back(f.index.at(PySequence_Fast_GET_ITEM(seq, i)));
        Py_DECREF(seq);
    }
    std::vector<int32_t> tname, tsize;
    PyObject* tseq = PySequence_Fast(tables, "tables");
    if (!tseq) return nullptr;
    for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(tseq); i++) {
        PyObject* t = PySequence_Fast_GET_ITEM(tseq, i);
        int32_t s;
        if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 2 || !str_of(PyTuple_GET_ITEM(t, 0), f, s)) {
            Py_DECREF(tseq);
            if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "tables: (name, size) pairs");
            return nullptr;
        }
        tname.push_back(s);
        tsize.push_back((int32_t)PyLong_AsLong(PyTuple_GET_ITEM(t, 1)));
    }
    Py_DECREF(tseq);
    if (PyErr_Occurred()) return nullptr;
    mgc_input in;
    std::memset(&in, 0, sizeof in);
    in.n_nodes = (int32_t)f.op.size();
    in.op = f.op.data(); in.sort = f.sort.data(); in.width = f.width.data(); in.dom = f.dom.data();
    in.id = f.id.data(); in.arg_off = f.arg_off.data(); in.args = f.args.data();
    in.p0 = f.p0.data(); in.p1 = f.p1.data(); in.str = f.str.data(); in.cval_off = f.cval_off.data();
    in.cval = f.cval.data(); in.strings = f.strings.data(); in.n_strings = f.n_strings;
    in.n_cons = (int32_t)ci.size(); in.cons = ci.data();
    in.n_probes = (int32_t)pi.size(); in.probes = pi.data();
    in.n_tables = (int32_t)tname.size(); in.table_name = tname.data(); in.table_size = tsize.data();
    in.default_entries = default_entries; in.nreg = nreg;
    in.n_extra = (int32_t)(PyBytes_GET_SIZE(extra) / 32);
    in.extra = (const uint32_t*)PyBytes_AS_STRING(extra);
    in.leaf_pools = leaf_pools; in.const_keys = const_keys; in.solve = solve;
    in.remat_mode = remat_mode; in.remat_k = remat_k; in.keep_clean = keep_clean;
    in.search_hints = search_hints; in.abi_presets = abi_presets;
    in.n_cval = (int32_t)f.cval.size(); in.n_string_bytes = (int32_t)f.strings.size();
    mgc_result* res = nullptr;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = mgc_compile(&in, &res);
    Py_END_ALLOW_THREADS
    PyObject* out;
    if (rc != MGC_OK) {
        out = Py_BuildValue("(isOOiO)", rc, mgc_error(res), Py_None, Py_None, 0, Py_None);
    } else {
        int32_t n_ins, rows, ncv;
        const uint32_t* code = mgc_code(res, &n_ins);
        const uint32_t* table = mgc_table(res, &rows, &ncv);
        static const char empty[1] = {0};            // y# turns a NULL buffer into None
        out = Py_BuildValue("(iOy#y#is)", rc, Py_None, code ? (const char*)code : empty,
                            (Py_ssize_t)(16 * n_ins), table ? (const char*)table : empty,
                            (Py_ssize_t)(32 * rows), ncv, mgc_meta(res));
    }
    mgc_free(res);
    return out;
}

// _mythcc.buckets(constraints) -> (group label per constraint (labels in
// order of first occurrence), DAG nodes per group (symbol-bearing nodes of
// the group; 1 for a symbol-free constraint) — the compile-cost estimate of
// model.gpu_search): constraints share a group iff they share a
// free symbol — a variable by name, an array / uninterpreted function by
// name (mythril_amd/model.py dependence_buckets, the reference's
// IndependenceSolver DependenceMap, independence_solver.py:38-84).  One
// union-find over the DAG: a node joins each operand that holds a symbol,
// and every symbol node joins its name.
struct UF {
    std::vector<int> p;
    int add() { p.push_back((int)p.size()); return (int)p.size() - 1; }
    int find(int x) { while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; } return x; }
    void join(int a, int b) { a = find(a); b = find(b); if (a != b) p[b] = a; }
};

PyObject* py_buckets(PyObject*, PyObject* a) {
    PyObject* cons;
    if (!PyArg_ParseTuple(a, "O", &cons)) return nullptr;
    PyObject* seq = PySequence_Fast(cons, "constraints");
    if (!seq) return nullptr;
    std::unordered_map<PyObject*, int> idx;        // node -> UF element
    std::vector<char> has_sym;
    std::unordered_map<std::string, int> sym;      // "v:name" / "t:name" -> UF element
    UF uf;
    struct It { PyObject* node; PyObject* args; Py_ssize_t next; };
    std::vector<It> stack;
    auto fail = [&]() -> PyObject* {
        for (auto& it : stack) Py_DECREF(it.args);
        Py_DECREF(seq);
        return nullptr;
    };
    auto open = [&](PyObject* n) -> bool {
        PyObject* args = attr(n, s_args);
        if (!args) return false;
        PyObject* fs = PySequence_Fast(args, "args");
        Py_DECREF(args);
        if (!fs) return false;
        stack.push_back({n, fs, 0});
        return true;
    };
    auto close = [&](PyObject* n, PyObject* args) -> bool {
        int me = uf.add();
        has_sym.push_back(0);
        PyObject* op = attr(n, s_op);
        if (!op) return false;
        bool is_var = PyUnicode_CompareWithASCIIString(op, "var") == 0;
        bool is_tab = !is_var && (PyUnicode_CompareWithASCIIString(op, "array") == 0 ||
                                  PyUnicode_CompareWithASCIIString(op, "apply") == 0);
        Py_DECREF(op);
        if (is_var || is_tab) {
            PyObject* params = attr(n, s_params);
            if (!params) return false;
            PyObject* name = PyTuple_Check(params) && PyTuple_GET_SIZE(params) ? PyTuple_GET_ITEM(params, 0) : nullptr;
            Py_ssize_t len;
            const char* s = name ? PyUnicode_AsUTF8AndSize(name, &len) : nullptr;
            if (!s) { Py_DECREF(params); if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "symbol name"); return false; }
            std::string key = std::string(is_var ? "v:" : "t:") + std::string(s, (size_t)len);
            Py_DECREF(params);
            auto it = sym.find(key);
            int se;
            if (it == sym.end()) {
                se = uf.add();
                has_sym.push_back(1);
                sym.emplace(key, se);
            } else {
                se = it->second;
            }
            uf.join(se, me);
            has_sym[me] = 1;
        }
        for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(args); i++) {
            int c = idx.at(PySequence_Fast_GET_ITEM(args, i));
            if (has_sym[c]) { uf.join(me, c); has_sym[me] = 1; }
        }
        idx.emplace(n, me);
        return true;
    };
    Py_ssize_t nc = PySequence_Fast_GET_SIZE(seq);
    for (Py_ssize_t i = 0; i < nc; i++) {
        PyObject* r = PySequence_Fast_GET_ITEM(seq, i);
        if (idx.count(r)) continue;
        if (!open(r)) return fail();
        while (!stack.empty()) {
            It& it = stack.back();
            if (it.next < PySequence_Fast_GET_SIZE(it.args)) {
                PyObject* c = PySequence_Fast_GET_ITEM(it.args, it.next++);
                if (idx.count(c)) continue;
                if (!open(c)) return fail();
                continue;
            }
            PyObject* n = it.node;
            PyObject* args = it.args;
            stack.pop_back();
            bool ok = close(n, args);
            Py_DECREF(args);
            if (!ok) return fail();
        }
    }
    PyObject* out = PyList_New(nc);
    std::unordered_map<int, long> label;
    std::unordered_map<int, long> per_root;           // symbol-bearing nodes per set
    for (auto& kv : idx) if (has_sym[kv.second]) per_root[uf.find(kv.second)]++;
    std::vector<long> sizes;
    for (Py_ssize_t i = 0; i < nc; i++) {
        int e = idx.at(PySequence_Fast_GET_ITEM(seq, i));
        long l;
        if (!has_sym[e]) {
            l = (long)label.size();
            label[-1 - (int)i] = l;                     // symbol-free: a group of its own
            sizes.push_back(1);
        } else {
            int root = uf.find(e);
            auto it = label.find(root);
            if (it == label.end()) {
                l = label[root] = (long)label.size();
                sizes.push_back(per_root[root]);
            } else {
                l = it->second;
            }
        }
        PyList_SET_ITEM(out, i, PyLong_FromLong(l));
    }
    Py_DECREF(seq);
    PyObject* sz = PyList_New((Py_ssize_t)sizes.size());
    for (size_t g = 0; g < sizes.size(); g++) PyList_SET_ITEM(sz, (Py_ssize_t)g, PyLong_FromLong(sizes[g]));
    return Py_BuildValue("(NN)", out, sz);
}

PyMethodDef methods[] = {
    {"compile", py_compile, METH_VARARGS, "Flatten a constraint DAG and compile it (include/mythcc.h)."},
    {"buckets", py_buckets, METH_VARARGS, "Independent-group label of each constraint."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mythcc", "native host compiler front-end", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__mythcc(void) {
    s_op = PyUnicode_InternFromString("op");
    s_sort = PyUnicode_InternFromString("sort");
    s_width = PyUnicode_InternFromString("width");
    s_dom = PyUnicode_InternFromString("dom");
    s_args = PyUnicode_InternFromString("args");
    s_params = PyUnicode_InternFromString("params");
    s_id = PyUnicode_InternFromString("id");
    s_enc = PyUnicode_InternFromString("_enc");
    return PyModule_Create(&module);
}
