"""bench.py with module attributes overridden first (same-process A/B of switches that are not environment knobs):

    python tools/bench_with.py ops.hip._Q8_ONLY=False -- --model roberta-large --task masked-lm --dtype fp8 ...

Each ``path.attr=value`` sets ``huggingface_sagemaker_tensorflow_distributed_amd.<path>.<attr> = eval(value)``
(path: a module, or a module then attributes, e.g. ``train.trainer.Trainer.zero_grad_in_optimizer``)."""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
argv = sys.argv[1:]
sep = argv.index("--") if "--" in argv else len(argv)
for spec in argv[:sep]:
    path, val = spec.split("=", 1)
    parts = path.split(".")
    # the longest importable module prefix, then attributes (a class attribute: train.trainer.Trainer.attr)
    for i in range(len(parts) - 1, 0, -1):
        try:
            obj = importlib.import_module("huggingface_sagemaker_tensorflow_distributed_amd." + ".".join(parts[:i]))
            break
        except ModuleNotFoundError:
            continue
    for name in parts[i:-1]:
        obj = getattr(obj, name)
    setattr(obj, parts[-1], eval(val))
    print(f"[bench_with] {path} = {val}", file=sys.stderr)
sys.argv = [os.path.join(ROOT, "bench.py")] + argv[sep + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
