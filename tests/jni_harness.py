"""Calls the JNI shim (java/jni/hgx_jni.c) the way a JVM would, without a JVM.  TEST INFRASTRUCTURE.

`tests/native/build/libhgx_jni_harness.so` is the shim linked with a test JNIEnv
(`tests/native/fake_jni.c`).  The native signatures are read from `Hgx.java` itself, so a call here
passes exactly the Java argument list the declaration has (a drifted declaration fails to bind).
Each call:
  - converts Python arguments to Java objects (numpy / lists -> int[] / long[] / byte[], str -> String,
    None -> null); a writable contiguous numpy array of the Java element type gets back what the native
    committed to its Java copy (Java arrays are passed by reference);
  - calls `Java_org_hypergraphdb_gpu_Hgx_<name>(env, clazz, ...)`;
  - checks the JNI discipline the fake env records (pins all released, inputs unmodified, no JNI call
    with an exception pending);
  - raises `JavaException(class, message)` when the native left an exception pending, else returns the
    result converted back (arrays -> numpy copies, String -> str).
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "build", "libhgx_jni_harness.so")
HGX_JAVA = os.path.join(ROOT, "java", "org", "hypergraphdb", "gpu", "Hgx.java")

_SCALAR = {"long": C.c_int64, "int": C.c_int32, "boolean": C.c_uint8, "double": C.c_double}
_KIND = {"int[]": (0, np.int32), "long[]": (1, np.int64), "byte[]": (2, np.int8), "double[]": (3, np.float64)}


class JavaException(Exception):
    def __init__(self, cls: str, msg: str):
        super().__init__(f"{cls}: {msg}")
        self.cls = cls.replace("/", ".")
        self.msg = msg


class JniViolation(AssertionError):
    pass


def java_natives() -> dict:
    """name -> (return type, [parameter types]) of every `static native` in Hgx.java."""
    src = open(HGX_JAVA).read()
    out = {}
    for ret, name, params in re.findall(r"static native ([\w\[\]]+) (\w+)\(([^)]*)\)", src, re.S):
        types = [p.strip().rsplit(None, 1)[0] for p in params.split(",") if p.strip()]
        out[name] = (ret, types)
    return out


class Jni:
    """One JNIEnv (one 'Java thread').  `jni.<native>(*args)` calls that native."""

    def __init__(self):
        self.L = C.CDLL(LIB)
        L = self.L
        L.fj_env_new.restype = C.c_void_p
        L.fj_env_free.argtypes = [C.c_void_p]
        L.fj_new_array.restype = C.c_void_p
        L.fj_new_array.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
        L.fj_new_string.restype = C.c_void_p
        L.fj_new_string.argtypes = [C.c_void_p, C.c_char_p]
        L.fj_kind.argtypes = [C.c_void_p]
        L.fj_length.restype = C.c_int64
        L.fj_length.argtypes = [C.c_void_p]
        L.fj_data.restype = C.c_void_p
        L.fj_data.argtypes = [C.c_void_p]
        L.fj_release.argtypes = [C.c_void_p, C.c_void_p]
        for f in ("fj_exception_class", "fj_exception_message", "fj_violation_text"):
            getattr(L, f).restype = C.c_char_p
            getattr(L, f).argtypes = [C.c_void_p]
        L.fj_exception_clear.argtypes = [C.c_void_p]
        L.fj_outstanding_pins.restype = C.c_int64
        L.fj_outstanding_pins.argtypes = [C.c_void_p]
        L.fj_violations.argtypes = [C.c_void_p]
        L.fj_inject_oom.argtypes = [C.c_void_p, C.c_int64]
        L.fj_live_objects.restype = C.c_int64
        L.fj_live_objects.argtypes = [C.c_void_p]
        self.env = L.fj_env_new()
        self.natives = java_natives()
        self.called: set[str] = set()
        self._fns = {}

    def close(self):
        if self.env:
            self.L.fj_env_free(self.env)
            self.env = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- objects ----
    def _to_java(self, jtype: str, v):
        if v is None:
            return None
        if jtype == "String":
            return self.L.fj_new_string(self.env, str(v).encode())
        kind, dt = _KIND[jtype]
        a = np.ascontiguousarray(np.asarray(v, dtype=dt))
        return self.L.fj_new_array(self.env, kind, a.ctypes.data if a.size else None, a.size)

    def _from_java(self, jtype: str, o):
        if not o:
            return None
        if jtype == "String":
            n = self.L.fj_length(o)
            s = C.string_at(self.L.fj_data(o), n).decode()
        else:
            kind, dt = _KIND["double[]" if jtype == "jarray_double" else jtype]
            n = self.L.fj_length(o)
            s = np.ctypeslib.as_array(C.cast(self.L.fj_data(o), C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                      (n,)).copy() if n else np.zeros(0, dt)
        self.L.fj_release(self.env, o)
        return s

    def inject_oom(self, nth: int):
        self.L.fj_inject_oom(self.env, nth)

    def live_objects(self) -> int:
        return self.L.fj_live_objects(self.env)

    # ---- calls ----
    def _fn(self, name):
        if name not in self._fns:
            ret, params = self.natives[name]
            f = getattr(self.L, f"Java_org_hypergraphdb_gpu_Hgx_{name}")
            f.argtypes = [C.c_void_p, C.c_void_p] + [_SCALAR.get(t, C.c_void_p) for t in params]
            f.restype = None if ret == "void" else _SCALAR.get(ret, C.c_void_p)
            self._fns[name] = f
        return self._fns[name]

    def call(self, name: str, *args):
        ret, params = self.natives[name]
        if len(args) != len(params):
            raise TypeError(f"Hgx.{name} takes {len(params)} arguments ({', '.join(params)}), got {len(args)}")
        jargs = []
        for t, v in zip(params, args):
            if t in _SCALAR:
                jargs.append(int(v) if t != "double" else float(v))
            else:
                jargs.append(self._to_java(t, v))
        self.called.add(name)
        r = self._fn(name)(self.env, None, *jargs)
        for t, v, o in zip(params, args, jargs):   # the "Java" inputs go out of scope
            if t not in _SCALAR and o:
                if t in _KIND and isinstance(v, np.ndarray) and v.size and v.flags.writeable and \
                        v.flags.c_contiguous and v.dtype == _KIND[t][1]:
                    # Java arrays are passed by reference: what the native committed is the caller's
                    v[...] = np.ctypeslib.as_array(
                        C.cast(self.L.fj_data(o), C.POINTER(np.ctypeslib.as_ctypes_type(v.dtype))), (v.size,)
                    ).reshape(v.shape)
                self.L.fj_release(self.env, o)
        L = self.L
        pins = L.fj_outstanding_pins(self.env)
        if L.fj_violations(self.env) or pins:
            raise JniViolation(f"Hgx.{name}: {L.fj_violation_text(self.env).decode()} (outstanding pins: {pins})")
        cls = L.fj_exception_class(self.env)
        if cls:
            msg = L.fj_exception_message(self.env).decode()
            L.fj_exception_clear(self.env)
            if r and ret not in _SCALAR and ret != "void":
                raise JniViolation(f"Hgx.{name} returned an object with an exception pending")
            raise JavaException(cls.decode(), msg)
        if ret == "void":
            return None
        if ret in _SCALAR:
            return r
        # `jarray` returns of double[] are declared double[] in Java
        return self._from_java(ret, r)

    def __getattr__(self, name):
        if name.startswith("_") or name not in self.__dict__.get("natives", {}):
            raise AttributeError(name)
        return lambda *a: self.call(name, *a)
