"""tools/traffic_parse.py names every kernel of a profiled step (bytes
landed under '' and template fragments because '(anonymous namespace)' and template
arguments were cut at the wrong parenthesis)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from traffic_parse import kernel_short_name  # noqa: E402

NAMES = {
    "(anonymous namespace)::inflate2_kernel((anonymous namespace)::Item const*, unsigned int const*, unsigned int*, "
    "int*, unsigned int*, unsigned int const*, hz2::Tune, unsigned char*)": "inflate2_kernel",
    "(anonymous namespace)::copy_kernel(unsigned char const*, unsigned char*, (anonymous namespace)::CopyDesc const*,"
    " long)": "copy_kernel",
    "void at::native::elementwise_kernel<128, 4, at::native::gpu_kernel_impl_nocast<at::native::FillFunctor<int> >"
    "(at::TensorIteratorBase&, at::native::FillFunctor<int> const&)::{lambda(int)#1}>(int, "
    "at::native::gpu_kernel_impl_nocast<at::native::FillFunctor<int> >(at::TensorIteratorBase&, "
    "at::native::FillFunctor<int> const&)::{lambda(int)#1})": "elementwise_kernel",
    "void at::native::vectorized_elementwise_kernel<4, at::native::FillFunctor<int>, at::detail::Array<char*, 1ul> >"
    "(int, at::native::FillFunctor<int>, at::detail::Array<char*, 1ul>)": "vectorized_elementwise_kernel",
    "void at::native::(anonymous namespace)::direct_copy_kernel_cuda(at::TensorIteratorBase&)": "direct_copy_kernel_cuda",
    "__amd_rocclr_copyBuffer": "__amd_rocclr_copyBuffer",
    "plan_descs_kernel(long const*, long)": "plan_descs_kernel",
}


def test_kernel_short_names():
    for full, short in NAMES.items():
        assert kernel_short_name(full) == short, full


def test_cfg3_attribution_names_every_kernel(tmp_path):
    for d, counter, base in (("fetch3", "FETCH_SIZE", 1000.0), ("write3", "WRITE_SIZE", 10.0)):
        p = tmp_path / d / "x"
        p.mkdir(parents=True)
        with open(p / "fetch_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for i, full in enumerate(NAMES):
                w.writerow({"Dispatch_Id": i, "Kernel_Name": full, "Counter_Name": counter, "Counter_Value": base})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_parse.py"), str(tmp_path), "r4",
                          "cfg3"], capture_output=True, text=True, check=True).stdout
    res = json.loads(out)
    assert set(res["per_kernel_fetch_write_bytes"]) == set(NAMES.values())
    assert "" not in res["per_kernel_fetch_write_bytes"]
