"""Tool-only probe builds of the product library (never shipped; wrong numerics by design):
one LDS update swapped, to find what bounds a kernel.
  nolds: forward, no LDS update (a never-true branch keeps the loads and products alive)
  u64:   forward, ds_add_u64 of the f64 bits (the integer LDS atomic rate)
  rmw:   forward, plain read-add-write (ds_read_b64 + ds_write_b64, racy)
  bnolds: backward (sspmm_bwd4, CAS pairs), no compare-and-swap (the reads stay)
  bu32:   backward, two ds_add_u32 of the float bits per pair instead of the CAS
Writes tools/libmaxk_probe_<name>.so; select one with MAXK_HIP_LIB=... (maxk_kernels/_lib.py).
  python tools/probe_fwd_build.py [names...]"""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "spgemm-gnn_amd")
ORIG = "    lds_add(p, (double)v);\n  }\n};"
BODIES = {
    "nolds": "    if (__builtin_expect(v == 1234.5f, 0)) lds_add(p, (double)v);\n  }\n};",
    "u64": ("    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p),\n"
            "        (unsigned long long)__double_as_longlong((double)v), __ATOMIC_RELAXED,\n"
            "        __HIP_MEMORY_SCOPE_WORKGROUP);\n  }\n};"),
    "rmw": "    *p += (double)v;\n  }\n};",
}
BWD_ORIG = """          if (ok[u]) {
            u64 expected = old2[u][h];
            __hip_atomic_compare_exchange_strong(a + h, &expected,"""
BWD = {
    "bnolds": BWD_ORIG.replace("if (ok[u]) {", "if (ok[u] && x[u][2 * h] == 1234.5f) {"),
    "bu32": """          if (ok[u]) {
            __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(a + h), __float_as_uint(x[u][2 * h]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(a + h) + 1,
                                   __float_as_uint(x[u][2 * h + 1]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          if (false) {
            u64 expected = old2[u][h];
            __hip_atomic_compare_exchange_strong(a + h, &expected,""",
}
SRCS = ["maxk_topk.hip", "spgemm.hip", "plan.hip", "capi.cpp"]


def build(name):
    tmp = tempfile.mkdtemp(prefix="maxk_probe_")
    try:
        src = os.path.join(tmp, "csrc")
        shutil.copytree(os.path.join(PKG, "csrc"), src)
        p = os.path.join(src, "spgemm.hip")
        s = open(p).read()
        if name in BWD:
            assert s.count(BWD_ORIG) == 1, "sspmm_bwd4 CAS-pair block changed"
            s = s.replace(BWD_ORIG, BWD[name])
        else:
            assert s.count(ORIG) == 1, "LdsAcc<MAXK_ACC_F64>::add body changed"
            s = s.replace(ORIG, BODIES[name])
        open(p, "w").write(s)
        objs = []
        for f in SRCS:
            o = os.path.join(tmp, f + ".o")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                            "-I" + os.path.join(ROOT, "include"), "-I" + src, "-munsafe-fp-atomics",
                            "-c", os.path.join(src, f), "-o", o], check=True)
            objs.append(o)
        out = os.path.join(HERE, f"libmaxk_probe_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", *objs,
                        "-o", out], check=True)
        print(out)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(BODIES) + list(BWD):
        build(n)
