"""The built gfx950 code object: every product kernel runs without scratch (register spills go
to scratch memory, one round trip per spilled value; the conv in particular is register-bound,
DESIGN.md §5). Reads the kernel descriptors' metadata from libuttt_engine.so with the ROCm
LLVM tools; no GPU needed."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd", "libuttt_engine.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# product kernels (mangled-name fragments); the conv's ablation/diagnostic instances are not product
PRODUCT = {
    "k_wino3h_conv<residual>": "k_wino3h_convILb1ELi0ELi3E",
    "k_wino3h_conv<plain>": "k_wino3h_convILb0ELi0ELi3E",
    "k_select<cpp>": "8k_selectILb0E",
    "k_select<py>": "8k_selectILb1E",
    "k_apply": "7k_applyE",
    "k_scan": "6k_scanE",
    "k_move_end": "10k_move_endE",
    "k_finalize": "10k_finalizeE",
    "k_stem": "6k_stemE",
    "k_heads": "7k_headsE",
}


def kernel_metadata(tmp_path):
    fb = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fb}", LIB], check=True, capture_output=True)
    # one offload bundle per linked source file (engine, nn_kernels, wino3h_conv), concatenated
    data = fb.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    assert starts, "no offload bundle in .hip_fatbin"
    notes = ""
    for i, a in enumerate(starts):
        part, co = tmp_path / f"bundle{i}.bin", tmp_path / f"gfx950_{i}.o"
        part.write_bytes(data[a:starts[i + 1] if i + 1 < len(starts) else len(data)])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                       check=True, capture_output=True)
        notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                                text=True).stdout
    meta = {}
    # one YAML map per kernel in amdhsa.kernels; its keys are sorted, .name before .private_segment_fixed_size
    for block in re.split(r"\n\s+- \.", notes):
        name = re.search(r"\.name:\s+(\S+)", block)
        priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
        if name and priv:
            meta[name.group(1)] = int(priv.group(1))
    return meta


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-readelf")),
                    reason="library not built or ROCm LLVM tools missing")
def test_product_kernels_use_no_scratch(tmp_path):
    meta = kernel_metadata(tmp_path)
    for label, frag in PRODUCT.items():
        hits = {k: v for k, v in meta.items() if frag in k}
        assert hits, f"{label} not found in the code object"
        for k, v in hits.items():
            assert v == 0, f"{label} ({k}) uses {v} bytes of scratch (register spills)"
