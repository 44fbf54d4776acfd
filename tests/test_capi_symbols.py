"""CPU checks of the drop-in boundary: libtbe.so loads (no GPU needed to dlopen) and
exports every function include/*.h declares; the ctypes struct matches the header."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("tbe.h", "tbe_tools.h", "tbe_cluster.h", "tbe_strdir.h")]


def declared_functions(headers=HEADERS):
    names = []
    for h in headers:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^[a-z_][\w \*]*?\b(tbe_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for required in ("tbe_create", "tbe_destroy", "tbe_acquire_batch", "tbe_acquire_batch_device",
                     "tbe_query", "tbe_last_error", "tbe_synchronize", "tbe_gen_batch_device"):
        assert required in names


def test_library_exports_every_declared_symbol(engine_lib):
    lib = ctypes.CDLL(engine_lib)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    exported = subprocess.run(["nm", "-D", "--defined-only", engine_lib], capture_output=True,
                              text=True).stdout
    for n in declared_functions():
        assert re.search(rf"\bT {n}$", exported, flags=re.M), n


def test_python_binding_covers_header(engine_lib):
    from distributedratelimiting.redis_amd import _capi
    tbe_h = declared_functions(HEADERS[:1])   # the engine ABI; tbe_tools.h are test/bench helpers
    assert sorted(_capi.EXPORTED) == sorted(tbe_h)


def test_config_struct_layout(engine_lib, tmp_path):
    """ctypes TbeConfig must match the C compiler's layout of tbe_config."""
    from distributedratelimiting.redis_amd import _capi
    fields = [f[0] for f in _capi.TbeConfig._fields_]
    prog = tmp_path / "layout.c"
    body = "".join(f'printf("%zu\\n", offsetof(tbe_config, {f}));' for f in fields)
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tbe.h"\n'
                    'int main(void){' + body + 'printf("%zu\\n", sizeof(tbe_config));return 0;}')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(prog)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [getattr(_capi.TbeConfig, f).offset for f in fields] + [ctypes.sizeof(_capi.TbeConfig)]
    assert got == want


def test_fill_rate_matches_oracle(engine_lib):
    from distributedratelimiting.redis_amd import _capi
    from oracle.semantics import fill_rate_per_second
    lib = _capi.load()
    for tokens, ticks in [(1, 10_000_000), (10, 1_000_000), (3, 70_000_001), (7, 1)]:
        assert lib.tbe_fill_rate(tokens, ticks) == fill_rate_per_second(tokens, ticks)


def test_gpu_code_object_targets_gfx950(engine_lib):
    blob = open(engine_lib, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_integration_binds_every_engine_entry_point():
    """INTEGRATION.md's C# binding (the reference-side P/Invoke a maintainer adds) has a
    LibraryImport for every function include/tbe.h declares."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    bound = set(re.findall(r'EntryPoint = "(tbe_\w+)"', doc))
    missing = [n for n in declared_functions(HEADERS[:1]) if n not in bound]
    assert not missing, missing
