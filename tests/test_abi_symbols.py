"""CPU: every C-ABI library loads (no GPU needed to load) and exports every function its header
in include/ declares; the drop-in codec exports exactly the reference's symbol list."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "liberasurecode_amd", "lib")

HEADERS = {
    "ecamd_host.h": "libecamd_host.so",
    "ecamd.h": "libecamd.so",
    "liberasurecode_rs_vand.h": "liberasurecode_rs_vand.so.1",
    "xor_code.h": "libXorcode.so.1",
}

# libXorcode.sym:1-5 of the reference
REF_XORCODE_SYMS = sorted("""init_xor_hd_code xor_code_encode xor_hd_decode xor_hd_fragments_needed
xor_reconstruct_one""".split())


def test_xorcode_exports_exactly_reference_symbols():
    assert exported(os.path.join(LIB, "libXorcode.so.1")) == REF_XORCODE_SYMS
    assert declared("xor_code.h") == REF_XORCODE_SYMS

# liberasurecode_rs_vand.sym:1-13 of the reference (the CI symbol contract, check-symbols.sh)
REF_RS_VAND_SYMS = sorted("""create_decoding_matrix deinit_liberasurecode_rs_vand
free_systematic_matrix gaussj_inversion init_liberasurecode_rs_vand is_identity_matrix is_missing
liberasurecode_rs_vand_decode liberasurecode_rs_vand_encode liberasurecode_rs_vand_reconstruct
make_systematic_matrix print_matrix square_matrix_multiply""".split())


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    names = re.findall(r"^[A-Za-z_][\w \t\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "defined")))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return sorted(l.split()[-1] for l in out.splitlines() if " T " in l)


@pytest.mark.parametrize("header,lib", sorted(HEADERS.items()))
def test_header_symbols_exported(header, lib):
    path = os.path.join(LIB, lib)
    C.CDLL(path)  # loads without a GPU
    names = declared(header)
    assert names, header
    missing = sorted(set(names) - set(exported(path)))
    assert not missing, missing


def test_rs_vand_exports_exactly_reference_symbols():
    assert exported(os.path.join(LIB, "liberasurecode_rs_vand.so.1")) == REF_RS_VAND_SYMS
    assert declared("liberasurecode_rs_vand.h") == REF_RS_VAND_SYMS


# liberasurecode.sym:1-28 of the reference: the frontend's export contract
REF_LIBERASURECODE_SYMS = sorted("""alloc_and_set_buffer get_backend_id get_backend_version
get_data_ptr_from_fragment get_fragment_partition get_libec_version is_invalid_fragment
is_invalid_fragment_header liberasurecode_backend_available liberasurecode_backend_instance_get_by_desc
liberasurecode_crc32_alt liberasurecode_decode liberasurecode_decode_cleanup liberasurecode_encode
liberasurecode_encode_cleanup liberasurecode_exit liberasurecode_fragments_needed
liberasurecode_get_aligned_data_size liberasurecode_get_fragment_metadata liberasurecode_get_fragment_size
liberasurecode_get_minimum_encode_size liberasurecode_get_version liberasurecode_init
liberasurecode_instance_create liberasurecode_instance_destroy liberasurecode_reconstruct_fragment
liberasurecode_verify_fragment_metadata liberasurecode_verify_stripe_metadata""".split())

SYM_FILES = {"liberasurecode.so.1": ("liberasurecode.sym", REF_LIBERASURECODE_SYMS),
             "liberasurecode_rs_vand.so.1": ("liberasurecode_rs_vand.sym", REF_RS_VAND_SYMS),
             "libXorcode.so.1": ("libXorcode.sym", REF_XORCODE_SYMS)}


def check_symbols_get(path):
    """check-symbols.sh:15-21 get(): `nm --dynamic --defined-only | cut -c18- | LC_COLLATE=C sort`
    -- every defined dynamic symbol with its type letter, so data symbols or linker extras would
    show up too."""
    out = subprocess.run(["nm", "--dynamic", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return sorted((l[17:] for l in out.splitlines() if l.strip()), key=lambda x: x.encode())


@pytest.mark.parametrize("lib", sorted(SYM_FILES))
def test_check_symbols_contract(lib):
    """The reference CI's symbol gate (check-symbols.sh check, :23-28) applied to the drop-ins:
    the listing equals the reference's .sym file line for line ("T name" x 28 / 13 / 5)."""
    sym, names = SYM_FILES[lib]
    want = ["T " + n for n in sorted(names, key=lambda x: x.encode())]
    assert check_symbols_get(os.path.join(LIB, lib)) == want
    ref = os.path.join("/root/reference", sym)
    if os.path.exists(ref):  # the build container: the embedded list is the reference's file
        assert [l for l in open(ref).read().splitlines() if l.strip()] == want


def test_soname():
    out = subprocess.run(["readelf", "-d", os.path.join(LIB, "liberasurecode_rs_vand.so.1")],
                         capture_output=True, text=True, check=True).stdout
    assert "[liberasurecode_rs_vand.so.1]" in out


def test_no_gpu_fails_loudly():
    """Without a HIP device the codec refuses to create a generator (instance_create then fails
    with -EBACKENDINITERR in the frontend); there is no silent CPU fallback."""
    code = ("import ctypes as C, os; l = C.CDLL(os.path.join(%r, 'liberasurecode_rs_vand.so.1'));"
            "l.make_systematic_matrix.restype = C.c_void_p;"
            "print('NULL' if not l.make_systematic_matrix(4, 2) else 'PTR')" % LIB)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=120)
    has_gpu = os.path.exists("/dev/kfd")
    if has_gpu:
        assert "PTR" in r.stdout
    else:
        assert "NULL" in r.stdout and "no HIP device" in r.stderr


@pytest.mark.parametrize("header,lib", [("ecamd.h", "libecamd.so"), ("ecamd_host.h", "libecamd_host.so"),
                                        ("ecamd_probe.h", "libecamd_probe.so")])
def test_extension_exports_only_its_c_abi(header, lib):
    """The device / host extension libraries export their C ABI and nothing else: the C++
    internals, kernel stubs and helpers stay local (version script abi/ecamd.map)."""
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB, lib)], capture_output=True,
                         text=True, check=True).stdout
    names = sorted(l.split()[-1] for l in out.splitlines() if l.split()[-2] in "TtWwDdBbRrVv")
    stray = [n for n in names if not n.startswith("ecamd_") and not n.startswith("_end")
             and n not in ("_edata", "__bss_start", "_fini", "_init")]
    assert not stray, stray[:20]
    assert set(n for n in names if n.startswith("ecamd_")) <= set(declared(header)) | set(
        declared("ecamd_host.h")), "exported but undeclared"
