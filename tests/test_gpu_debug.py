"""Debug build of the extension (SURVEY.md §5 'bounds-check debug builds'): ``HSD_DEBUG=1`` loads
``_C_debug.so`` (compiled with -DHSD_DEBUG: a device synchronisation after every launch, HSD_DASSERT
device checks, host-side index range checks). Runs in a child process so the release module of this
test session is untouched."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

SCRIPT = textwrap.dedent("""
    import torch
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import _ext
    C = _ext.load()
    assert C.__name__.endswith("_C_debug"), C.__name__
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
    cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=1)
    m = build_model(cfg, seed=0).cuda()
    store = FlatParamStore(m, torch.device("cuda", 0), compute_dtype=torch.bfloat16)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device="cuda")
    am = torch.ones_like(ids)
    m.train()
    m.rng.new_step(0)
    loss, _ = m(ids, attention_mask=am, labels=torch.zeros(2, dtype=torch.long, device="cuda"))
    loss.backward()
    torch.cuda.synchronize()
    bad = ids.clone()
    bad[0, 3] = cfg.vocab_size + 5
    try:
        m(input_ids=bad, attention_mask=am)
    except RuntimeError as e:
        assert "out of vocabulary range" in str(e), e
        print("DEBUG_OK")
    else:
        raise SystemExit("out-of-range id was not caught")
""")


def test_debug_build_checks_indices(gpu):
    env = dict(os.environ, HSD_DEBUG="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "DEBUG_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
