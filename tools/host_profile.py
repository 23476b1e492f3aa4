"""Host-side cost of one pipelined TRPO iteration: cProfile over bench.py's timed loop,
printed by own time (GPU waits show up in the readback calls)."""
import cProfile
import pstats
import sys

sys.argv = ["bench.py"] + sys.argv[1:]
sys.path.insert(0, ".")
import runpy  # noqa: E402

prof = cProfile.Profile()
prof.enable()
try:
    runpy.run_path("bench.py", run_name="__main__")
finally:
    prof.disable()
    st = pstats.Stats(prof, stream=sys.stderr)
    st.sort_stats("tottime").print_stats(45)
    st.print_callers("is_available")
    st.sort_stats("cumtime").print_stats("modular_rl_amd|bench.py", 40)
