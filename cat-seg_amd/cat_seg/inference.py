"""The evaluation loop: detectron2 `inference_on_dataset` (what `Trainer.test`, train_net.py:302,
runs per test dataset; a copy is at viz_atten.py:166-318).

Every rank feeds its shard of the loader (cat_seg.data.build_test_loader) through the model
under `torch.no_grad()` / eval mode, times the steady state after min(5, len - 1) warm-up
iterations (device-synchronised per iteration, as there), hands each batch to the evaluator,
and finally calls `evaluator.evaluate()`, which sums the per-rank confusion matrices over
torch.distributed (the gather of plain_train_net.py:136-146).
"""
from __future__ import annotations

import datetime
import logging
import time
from contextlib import ExitStack, contextmanager

import torch
import torch.distributed as dist
from torch import nn


@contextmanager
def inference_context(model: nn.Module):
    training = model.training
    model.eval()
    try:
        yield
    finally:
        model.train(training)


class DatasetEvaluators:
    """Fan one loop out to several evaluators (detectron2 DatasetEvaluators)."""

    def __init__(self, evaluators):
        self._evaluators = list(evaluators)

    def reset(self):
        for e in self._evaluators:
            e.reset()

    def process(self, inputs, outputs):
        for e in self._evaluators:
            e.process(inputs, outputs)

    def evaluate(self):
        results = {}
        for e in self._evaluators:
            r = e.evaluate()
            for k, v in (r or {}).items():
                if k in results:
                    raise KeyError(f"Different evaluators produce results with the same key {k}")
                results[k] = v
        return results


def inference_on_dataset(model, data_loader, evaluator, log_period_s: float = 5.0):
    log = logging.getLogger(__name__)
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    total = len(data_loader)
    log.info("Start inference on %d batches", total)
    if evaluator is None:
        evaluator = DatasetEvaluators([])
    elif isinstance(evaluator, (list, tuple)):
        evaluator = DatasetEvaluators(evaluator)
    evaluator.reset()
    num_warmup = min(5, total - 1)
    start = time.perf_counter()
    t_data = t_compute = t_eval = 0.0
    last_log = start
    with ExitStack() as stack:
        if isinstance(model, nn.Module):
            stack.enter_context(inference_context(model))
        stack.enter_context(torch.no_grad())
        t0 = time.perf_counter()
        for idx, inputs in enumerate(data_loader):
            t_data += time.perf_counter() - t0
            if idx == num_warmup:
                start = time.perf_counter()
                t_data = t_compute = t_eval = 0.0
            t1 = time.perf_counter()
            outputs = model(inputs)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            t_compute += time.perf_counter() - t1
            t2 = time.perf_counter()
            evaluator.process(inputs, outputs)
            t_eval += time.perf_counter() - t2
            n = idx + 1 - num_warmup * int(idx >= num_warmup)
            if time.perf_counter() - last_log > log_period_s and n > 0:
                last_log = time.perf_counter()
                eta = datetime.timedelta(seconds=int((last_log - start) / n * (total - idx - 1)))
                log.info("Inference done %d/%d. Dataloading: %.4f s/iter. Inference: %.4f s/iter. Eval: %.4f s/iter. "
                         "ETA=%s", idx + 1, total, t_data / n, t_compute / n, t_eval / n, eta)
            t0 = time.perf_counter()
    total_time = time.perf_counter() - start
    timed = max(total - num_warmup, 1)
    log.info("Total inference time: %s (%.6f s / iter per device, on %d devices)",
             datetime.timedelta(seconds=int(total_time)), total_time / timed, world)
    log.info("Total inference pure compute time: %s (%.6f s / iter per device, on %d devices)",
             datetime.timedelta(seconds=int(t_compute)), t_compute / timed, world)
    results = evaluator.evaluate()
    return results if results is not None else {}
