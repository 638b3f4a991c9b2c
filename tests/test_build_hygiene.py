"""build() decides by content: a library is reused only if the
digest of the sources, flags and compiler recorded next to it equals the digest of
what is on disk now and the library's own sha256 matches the record; mtimes do not
matter.  CPU only (no hipcc run: the digests are compared, not rebuilt)."""
import json
import os

import pytest

from modulations_amd import build as Bd


def _fake_tree(tmp_path):
    src = tmp_path / "a.hip"
    src.write_text("// kernel v1\n")
    lib = tmp_path / "liba.so"
    lib.write_bytes(b"\x7fELF fake library")
    deps = [str(src)]
    with open(str(lib) + ".build.json", "w") as f:
        json.dump({"src_sha256": Bd.source_digest(deps), "lib_sha256": Bd._file_sha(str(lib)), "flags": Bd.FLAGS}, f)
    return src, lib, deps


def test_current_library_is_reused(tmp_path):
    src, lib, deps = _fake_tree(tmp_path)
    assert Bd.is_current(str(lib), deps)


def test_edited_source_with_old_mtime_rebuilds(tmp_path):
    src, lib, deps = _fake_tree(tmp_path)
    st = os.stat(src)
    src.write_text("// kernel v2\n")
    os.utime(src, (st.st_atime, st.st_mtime - 3600))       # older than the library: mtime says "fresh"
    assert not Bd.is_current(str(lib), deps)


def test_touched_unchanged_sources_do_not_rebuild(tmp_path):
    src, lib, deps = _fake_tree(tmp_path)
    os.utime(src, None)                                     # newer than the library, same content
    assert Bd.is_current(str(lib), deps)


def test_replaced_library_rebuilds(tmp_path):
    src, lib, deps = _fake_tree(tmp_path)
    lib.write_bytes(b"\x7fELF another build")
    assert not Bd.is_current(str(lib), deps)


def test_missing_record_rebuilds(tmp_path):
    src, lib, deps = _fake_tree(tmp_path)
    os.remove(str(lib) + ".build.json")
    assert not Bd.is_current(str(lib), deps)


@pytest.mark.gpu
def test_shipped_libraries_match_the_tree():
    """On the GPU box: the libraries the GPU tests load are what the sources
    shipped beside them produce (no stale binary behind a fresh checkout)."""
    assert Bd.is_current(Bd.OUT, Bd.DEPS), "lib/libtdec.so is stale: run python -m modulations_amd.build"
    assert Bd.is_current(Bd.MODEM_OUT, Bd.MODEM_DEPS), "lib/libmodem.so is stale"
