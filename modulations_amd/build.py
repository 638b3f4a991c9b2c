"""Build the gfx950 HIP libraries in-tree: modulations_amd/lib/libtdec.so (turbo
decoder + soft demapper, include/tdec.h) and modulations_amd/lib/libmodem.so
(modem front-end, include/modem.h).

``python -m modulations_amd.build`` or ``modulations_amd.build.build()``.
hipcc cross-compiles for gfx950 without a GPU.  Flags that the numerics need:
  -ffp-contract=off                  no FMA contraction (the reference has none)
  -fno-gpu-flush-denormals-to-zero   IEEE f32 denormals, as numpy/numba
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "tdec_api.hip")
DEPS = [SRC, os.path.join(HERE, "csrc", "tdec_kernels.hip"), os.path.join(HERE, "csrc", "tdec_workload.hip"), os.path.join(HERE, "csrc", "npmath.hip"),
        os.path.join(HERE, "csrc", "tdec_spl.hip"), os.path.join(HERE, "csrc", "tdec_lowlat.hip"), os.path.join(HERE, "csrc", "tdec_frame.hip"),
        os.path.join(ROOT, "include", "tdec.h")]
OUT = os.path.join(HERE, "lib", "libtdec.so")
MODEM_SRC = os.path.join(HERE, "csrc", "modem_api.hip")
MODEM_DEPS = [MODEM_SRC, os.path.join(HERE, "csrc", "modem_kernels.hip"), os.path.join(HERE, "csrc", "npmath.hip"),
              os.path.join(ROOT, "include", "modem.h")]
MODEM_OUT = os.path.join(HERE, "lib", "libmodem.so")

FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-gpu-flush-denormals-to-zero", "-Wall", "-Wno-unused-value", "-Wno-unused-result"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def source_digest(deps, extra=()):
    """sha256 over the sources, the flags and the compiler version: the identity
    of a build.  hipcc output is not byte-reproducible (a rebuild of the same
    sources differs in a few dozen bytes of the offload bundle), so measurements
    (profiles/traffic.json) are keyed by this digest as well as by the .so hash."""
    h = hashlib.sha256()
    for d in deps:
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    h.update("\0".join([*FLAGS, *extra]).encode())
    try:
        v = subprocess.run([hipcc(), "--version"], capture_output=True, text=True).stdout
    except OSError:
        v = ""
    h.update(v.encode())
    return h.hexdigest()


def build_info(out):
    """The build record written next to a library by _build_one (None if absent)."""
    try:
        with open(out + ".build.json") as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _file_sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def is_current(out, deps, extra=()):
    """Whether `out` was built from exactly the current sources, flags and
    compiler: its build record's src_sha256 equals the digest of what is on disk
    now and its lib_sha256 equals the library itself.  Content, not mtimes: a
    checkout or a copy that refreshes every mtime must not keep a stale binary,
    and one that does not must not rebuild for nothing."""
    info = build_info(out)
    if not info or not os.path.exists(out):
        return False
    return info.get("src_sha256") == source_digest(deps, extra) and info.get("lib_sha256") == _file_sha(out)


def _build_one(src, deps, out, force, extra):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if not force and is_current(out, deps, extra):
        return out
    tmp = out + ".tmp"
    cmd = [hipcc(), *FLAGS, *extra, "-I", os.path.join(ROOT, "include"), "-o", tmp, src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"hipcc failed building {os.path.basename(out)}")
    os.replace(tmp, out)   # a reader never sees a half-written library
    with open(out + ".build.json", "w") as f:
        json.dump({"src_sha256": source_digest(deps, extra), "lib_sha256": _file_sha(out),
                   "flags": [*FLAGS, *extra]}, f, indent=1)
    return out


def build(force=False, extra=()):
    """Both libraries; returns the path of libtdec.so."""
    _build_one(MODEM_SRC, MODEM_DEPS, MODEM_OUT, force, extra)
    return _build_one(SRC, DEPS, OUT, force, extra)


def build_modem(force=False):
    return _build_one(MODEM_SRC, MODEM_DEPS, MODEM_OUT, force, ())


def build_variant(name, defines):
    """Side-by-side variant for A/B timing (lib/libtdec_<name>.so).  Built on
    demand for one measurement and deleted afterwards (remove_variants): the
    variants are not product libraries and are not pushed with the tree."""
    out = os.path.join(HERE, "lib", f"libtdec_{name}.so")
    cmd = [hipcc(), *FLAGS, *[f"-D{d}" for d in defines], "-I", os.path.join(ROOT, "include"), "-o", out, SRC]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"hipcc failed building {out}")
    return out


def remove_variants():
    """Delete every lib/libtdec_<name>.so A/B variant."""
    d = os.path.join(HERE, "lib")
    for f in os.listdir(d):
        if f.startswith("libtdec_") and f.endswith(".so"):
            os.remove(os.path.join(d, f))


if __name__ == "__main__":
    if "--remove-variants" in sys.argv:
        remove_variants()
    elif "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], sys.argv[i + 2:]))
    else:
        print(build(force="--force" in sys.argv))
