#!/usr/bin/env python3
"""Probe build (not product): the library with source patches applied to a temporary copy of the
product sources, as tools/ab/libtkv_NAME.so, for in-process A/B runs (tools/ab_wal.py).

    python tools/variant.py NAME PATCH [PATCH ...]

Patches:
  stamp     s_memtime stamps around the sections of the WAL sweep's region body, summed per section
            over every wave (export tkv_debug_wal_stamps; tools/wal_sweep_probe.py prints the shares)
  region5k  5 KiB regions and 16 waves per sweep workgroup (4 waves per SIMD)
  region7k  7 KiB regions and 12 waves per sweep workgroup (3 waves per SIMD)
  listpoll64  crc_list_lanes polls the other workgroups' flags every 64 step groups instead of 4
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = os.path.join(ROOT, "tinykvpp_amd", "csrc")


def region5k(s):
    def rep(x, y):
        assert s.count(x) == 1, x
        return s.replace(x, y)
    s = rep("constexpr std::uint32_t kRegion = 10240;", "constexpr std::uint32_t kRegion = 5120;")
    s = rep("constexpr unsigned kSweepWaves = 8; ", "constexpr unsigned kSweepWaves = 16; ")
    return s


def stamp(s):
    def rep(x, y):
        assert s.count(x) >= 1, x
        return s.replace(x, y)
    s = rep("template <bool FIXUP, typename P>\n__device__ __forceinline__ void sweep_wave(",
            "__device__ unsigned long long g_stamp[8];\n"
            "#define ST(i) { const unsigned long long _t = __builtin_amdgcn_s_memtime(); tacc[i] += _t - tprev; tprev = _t; }\n"
            "template <bool FIXUP, typename P>\n__device__ __forceinline__ void sweep_wave(")
    s = rep("  constexpr P kNo = kNoneP<P>;\n",
            "  constexpr P kNo = kNoneP<P>;\n  unsigned long long tacc[8] = {}; unsigned long long tprev = __builtin_amdgcn_s_memtime();\n")
    s = rep("  auto body = [&](std::uint32_t rr) -> bool {\n    {\n", "  auto body = [&](std::uint32_t rr) -> bool {\n    {\n      ST(0); tacc[7] += 1;\n")
    s = rep("        Walk<P> wk;\n", "        ST(1);\n        Walk<P> wk;\n")
    s = rep("        walk_piece(win, rs, o, s, pe, size, true, wk);\n", "        walk_piece(win, rs, o, s, pe, size, true, wk);\n        ST(2);\n")
    s = rep("          // ---- 3. list and fold", "          ST(3);\n          // ---- 3. list and fold")
    s = rep("          for (std::uint32_t base = 0; base < nl; base += 64u) {", "          ST(4);\n          for (std::uint32_t base = 0; base < nl; base += 64u) {")
    s = rep("          if (bad_k != 0xFFFFFFFFu) Bpos", "          ST(5);\n          if (bad_k != 0xFFFFFFFFu) Bpos")
    s = rep("      e = next_e;\n", "      ST(6);\n      e = next_e;\n")
    s = rep("  if (!FIXUP && lane == 0) a.l_cnt[wave]",
            "  if (lane == 0) for (int i = 0; i < 8; ++i) atomicAdd(&g_stamp[i], tacc[i]);\n  if (!FIXUP && lane == 0) a.l_cnt[wave]")
    s += ("\nextern \"C\" int tkv_debug_wal_stamps(unsigned long long* out) {\n"
          "  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tkv::g_stamp), 64) != hipSuccess) return -1;\n"
          "  unsigned long long z[8] = {};\n"
          "  return hipMemcpyToSymbol(HIP_SYMBOL(tkv::g_stamp), z, 64) == hipSuccess ? 0 : -1;\n}\n")
    return s


def region7k(s):
    s = s.replace("constexpr std::uint32_t kRegion = 10240;", "constexpr std::uint32_t kRegion = 7168;")
    return s.replace("constexpr unsigned kSweepWaves = 8; ", "constexpr unsigned kSweepWaves = 12; ")


def listpoll64(s):
    x = "if (nchk++ % 4u == 0u) {"
    assert s.count(x) == 1
    return s.replace(x, "if (nchk++ % 64u == 0u) {")


PATCHES = {"stamp": stamp, "region5k": region5k, "region7k": region7k, "listpoll64": listpoll64}


def main():
    name, patches = sys.argv[1], sys.argv[2:]
    t = tempfile.mkdtemp()
    try:
        src = os.path.join(t, "csrc")
        shutil.copytree(H, src, ignore=shutil.ignore_patterns("build", "*.so", "*.o"))
        for fn in ("tkv_wal_device.hip", "tkv_crc32_kernels.hip"):
            p = os.path.join(src, fn)
            with open(p) as f:
                s = f.read()
            for pn in patches:
                if (pn.startswith("list")) == (fn == "tkv_crc32_kernels.hip"):
                    s = PATCHES[pn](s)
            with open(p, "w") as f:
                f.write(s)
        p = os.path.join(src, "tkv_wal_device.hip")
        fl = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"), "-I" + src]
        hc = "/opt/rocm/bin/hipcc"
        subprocess.check_call([hc] + fl + ["-c", os.path.join(src, "tkv_crc32_kernels.hip"), "-o", os.path.join(t, "k.o")])
        subprocess.check_call([hc] + fl + ["-c", p, "-o", os.path.join(t, "w.o")])
        b = os.path.join(H, "build")
        objs = [os.path.join(b, n) for n in ("tkv_crc32_host.o", "tkv_formats.o", "tkv_crc32_span.o", "tkv_wal_records.o", "tkv_build_id.o")]
        os.makedirs(os.path.join(ROOT, "tools", "ab"), exist_ok=True)
        subprocess.check_call([hc, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", os.path.join(ROOT, "tools", "ab", "libtkv_%s.so" % name),
                               os.path.join(t, "k.o"), os.path.join(t, "w.o")] + objs + ["-lpthread"])
    finally:
        shutil.rmtree(t)


if __name__ == "__main__":
    main()
