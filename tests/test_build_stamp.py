"""build.py never relabels a stale library.

The stamp next to liblsp_hip.so names the sources it was linked from, and
bench.py matches PMC profiles to the benched build by it.  A source can change
without a newer mtime (a checkout, ``rsync -t``); build() must then recompile
and relink, not rewrite the stamp.  The test drives build() over a scratch
tree with a stand-in compiler (a script that writes a digest of its input to
its ``-o`` path), so it runs in a second and touches nothing in the repo.
"""
import hashlib
import os
import stat
import sys
import textwrap

import pytest

from linea_stark_prover_amd import build as B

FAKE_CC = textwrap.dedent("""\
    #!{py}
    import hashlib, sys
    a = sys.argv[1:]
    out = a[a.index("-o") + 1]
    srcs = [x for x in a if x.endswith((".cpp", ".hip"))]
    objs = [x for x in a if x.endswith(".o") and x != out]
    h = hashlib.sha256()
    for f in srcs + objs:
        h.update(open(f, "rb").read())
    with open(out, "w") as fh:
        fh.write(h.hexdigest())
    with open({log!r}, "a") as fh:
        fh.write(("link " if "-shared" in a else "compile ") + out + "\\n")
    """)


@pytest.fixture
def tree(tmp_path, monkeypatch):
    root = tmp_path
    (root / "include").mkdir()
    (root / "include" / "lsp.h").write_text("/* header */\n")
    csrc = root / "csrc"
    csrc.mkdir()
    (csrc / "a.cpp").write_text("int a() { return 1; }\n")
    (csrc / "b.hip").write_text("int b() { return 2; }\n")
    log = root / "cc.log"
    cc = root / "fakecc"
    cc.write_text(FAKE_CC.format(py=sys.executable, log=str(log)))
    cc.chmod(cc.stat().st_mode | stat.S_IEXEC)
    libdir = root / "_lib"
    monkeypatch.setattr(B, "ROOT", str(root))
    monkeypatch.setattr(B, "CSRC", str(csrc))
    monkeypatch.setattr(B, "BUILD", str(root / "_build"))
    monkeypatch.setattr(B, "LIBDIR", str(libdir))
    monkeypatch.setattr(B, "LIB", str(libdir / "lib.so"))
    monkeypatch.setattr(B, "SOURCES", ["a.cpp", "b.hip"])
    monkeypatch.setattr(B, "HIPCC", str(cc))
    return root, csrc, log


def _log(log):
    return log.read_text().splitlines() if log.exists() else []


def test_backdated_source_edit_rebuilds_not_relabels(tree):
    root, csrc, log = tree
    lib = B.build(verbose=False)
    assert B.library_hash() == B.source_hash()
    first = _log(log)
    assert sum(l.startswith("compile") for l in first) == 2 and first[-1].startswith("link")

    # nothing changed: no compile, no link
    B.build(verbose=False)
    assert _log(log) == first

    # edit a source, then back-date it below its object's mtime
    obj = os.path.join(B.BUILD, "a.o")
    old_obj = open(obj).read()
    old_lib = open(lib).read()
    src = csrc / "a.cpp"
    src.write_text("int a() { return 42; }\n")
    t = os.path.getmtime(obj) - 100
    os.utime(src, (t, t))
    assert B.library_hash() != B.source_hash()

    B.build(verbose=False)
    after = _log(log)[len(first):]
    assert any(l.startswith("compile") and l.endswith("a.o") for l in after), after
    assert after[-1].startswith("link")
    assert open(obj).read() != old_obj == hashlib.sha256(b"int a() { return 1; }\n").hexdigest()
    assert open(obj).read() == hashlib.sha256(src.read_bytes()).hexdigest()
    assert open(lib).read() != old_lib
    assert B.library_hash() == B.source_hash()


def test_missing_library_stamp_relinks(tree):
    """objects whose own stamps match their sources are kept; the library is
    relinked from them and stamped"""
    root, csrc, log = tree
    B.build(verbose=False)
    n = len(_log(log))
    os.remove(B.LIB + ".src")
    B.build(verbose=False)
    again = _log(log)[n:]
    assert [l.split()[0] for l in again] == ["link"]
    assert B.library_hash() == B.source_hash()


def test_header_edit_recompiles_everything(tree):
    root, csrc, log = tree
    B.build(verbose=False)
    n = len(_log(log))
    hdr = root / "include" / "lsp.h"
    t = os.path.getmtime(hdr)
    hdr.write_text("/* header, edited */\n")
    os.utime(hdr, (t - 100, t - 100))  # older than every object
    B.build(verbose=False)
    again = _log(log)[n:]
    assert sum(l.startswith("compile") for l in again) == 2 and again[-1].startswith("link")
    assert B.library_hash() == B.source_hash()
