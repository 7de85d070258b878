"""Print every segment of one (pixel, sample) path, from the GPU or from the oracle (diagnostic).

    ART_LIB=$PWD/another_raytracer_amd/libart_trace.so python tools/trace_path.py gpu SCENE W H PIXEL SAMPLE
    python tools/trace_path.py oracle SCENE W H PIXEL SAMPLE

The GPU side needs the ART_TRACE build (make -C another_raytracer_amd/csrc OUT=../libart_trace.so
OBJDIR=../../build/trace EXTRA=-DART_TRACE ../libart_trace.so); both sides print lines starting with TRACE in one
format (bit patterns of the ray, hit point, normal), so `diff` finds the first operation where they part.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    side, scene = sys.argv[1], sys.argv[2]
    W, H, pixel, sample = map(int, sys.argv[3:7])
    y = pixel // W
    if side == "gpu":
        os.environ["ART_TRACE"] = f"{pixel}:{sample}"
        from tests.test_gpu_parity import gpu_render
        # the band (1, H, y) is row y alone: one row of W pixels at sample + 1 samples
        gpu_render(scene, W, H, sample + 1, band=(1, H, y))
    else:
        os.environ["ORC_TRACE"] = f"{pixel}:{sample}"
        from tests.oracle_lib import oracle_render_rows
        oracle_render_rows(scene, W, H, sample + 1, [y], threads=1)
    sys.stdout.flush()


if __name__ == "__main__":
    main()
