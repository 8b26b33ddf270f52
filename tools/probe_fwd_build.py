"""Tool-only probe builds of the product library (never shipped; wrong numerics by design):
the forward's LDS update swapped, to find what bounds spgemm_fwd_kernel at each k.
  nolds: no LDS update (a never-true branch keeps the loads and products alive)
  u64:   ds_add_u64 of the f64 bits (the integer LDS atomic rate)
  rmw:   plain read-add-write (ds_read_b64 + ds_write_b64, racy)
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
SRCS = ["maxk_topk.hip", "spgemm.hip", "plan.hip", "capi.cpp"]


def build(name):
    tmp = tempfile.mkdtemp(prefix="maxk_probe_")
    try:
        src = os.path.join(tmp, "csrc")
        shutil.copytree(os.path.join(PKG, "csrc"), src)
        p = os.path.join(src, "spgemm.hip")
        s = open(p).read()
        assert s.count(ORIG) == 1, "LdsAcc<MAXK_ACC_F64>::add body changed"
        open(p, "w").write(s.replace(ORIG, BODIES[name]))
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
    for n in sys.argv[1:] or list(BODIES):
        build(n)
