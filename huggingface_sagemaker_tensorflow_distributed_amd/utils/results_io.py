"""Result files with the exact byte format of the reference.

* ``train_results.txt`` (``scripts/train.py:157-165``): one ``"%s = %s\\n" % (key, per_epoch_list)``
  line per Keras history key, then ``train_runtime = {'train_runtime': X}``. The MirroredStrategy
  script omits the runtime line (``scripts/singe_node_train.py:96-101``).
* ``eval_results.txt`` (``scripts/train.py:172-179``): one ``"%s = %s\\n" % (key, float)`` per metric.
"""
from __future__ import annotations

import logging
import os
from typing import Dict, List, Mapping, Optional

logger = logging.getLogger(__name__)


def write_train_results(output_dir: str, history: Mapping[str, List[float]],
                        train_runtime: Optional[Dict[str, float]] = None) -> str:
    os.makedirs(output_dir, exist_ok=True)
    path = os.path.join(output_dir, "train_results.txt")
    with open(path, "w") as writer:
        logger.info("***** Train results *****")
        for key, value in history.items():
            logger.info("  %s = %s", key, value)
            writer.write("%s = %s\n" % (key, value))
        if train_runtime is not None:
            writer.write(f"train_runtime = {train_runtime}\n")
    return path


def write_eval_results(output_dir: str, result: Mapping[str, float]) -> str:
    os.makedirs(output_dir, exist_ok=True)
    path = os.path.join(output_dir, "eval_results.txt")
    with open(path, "w") as writer:
        logger.info("***** Eval results *****")
        logger.info(dict(result))
        for key, value in result.items():
            logger.info("  %s = %s", key, value)
            writer.write("%s = %s\n" % (key, value))
    return path


def parse_results(path: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    with open(path) as f:
        for line in f:
            if " = " in line:
                k, v = line.rstrip("\n").split(" = ", 1)
                out[k] = v
    return out
