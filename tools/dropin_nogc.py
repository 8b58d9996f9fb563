import gc, runpy, sys
gc.disable()
sys.argv = ["dropin_latency.py", "--calls", "30", "--out", "gpurun_out/i24/dropin_nogc.json"]
runpy.run_path("tools/dropin_latency.py", run_name="__main__")
