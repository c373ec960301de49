"""Admission-time sharding of independent streams over the GPUs of a node.

SURVEY.md §8e: streams are independent (``src/recognizer.h:76-110``; the
reference batch pipeline keys everything by stream id,
``src/batch_recognizer.cc:167``), so the node shards them with no data-path
exchange.  The only collective is control traffic: once per scheduling epoch
every rank contributes its number of free stream slots (one int32) to an
all-gather (RCCL over xGMI with the ``nccl`` backend, gloo on CPU), and every
rank runs the same deterministic plan over the shared utterance queue, so
new utterances go to the GPUs with the most free capacity without any rank
sending audio or decoder state anywhere.  A GPU that drains its streams
faster simply receives more of the queue (work-stealing at admission).
"""
from __future__ import annotations


def plan_admission(free, queue_head, queue_len):
    """Assign queue entries [queue_head, queue_len) to ranks: each entry in
    order goes to the rank with the most free slots left (ties: lower rank).
    Returns (per-rank lists of queue indices, new queue head).  Pure and
    deterministic: every rank computes the same plan from the gathered
    counts."""
    left = list(free)
    out = [[] for _ in left]
    q = queue_head
    while q < queue_len:
        r = max(range(len(left)), key=lambda i: (left[i], -i))
        if left[r] <= 0:
            break
        out[r].append(q)
        left[r] -= 1
        q += 1
    return out, q


class AdmissionController:
    """Per-epoch admission over ``torch.distributed`` (one int32 per rank)."""

    def __init__(self, dist, queue_len, device="cpu"):
        self.dist = dist
        self.queue_len = queue_len
        self.head = 0
        self.device = device
        self.world = dist.get_world_size() if dist is not None else 1
        self.rank = dist.get_rank() if dist is not None else 0
        self.epochs = 0

    def admit(self, free_slots):
        """Collective: every rank calls it with its free slot count; returns
        the queue indices this rank admits now."""
        if self.dist is None:
            counts = [int(free_slots)]
        else:
            counts = [c[0] for c in self.gather([int(free_slots)])]
        plan, self.head = plan_admission(counts, self.head, self.queue_len)
        self.epochs += 1
        return plan[self.rank]

    def gather(self, values):
        """All-gather a short int32 vector per rank -> list over ranks."""
        if self.dist is None:
            return [list(values)]
        import torch
        mine = torch.tensor(values, dtype=torch.int32, device=self.device)
        allc = [torch.zeros_like(mine) for _ in range(self.world)]
        self.dist.all_gather(allc, mine)
        return [[int(x) for x in t.cpu().tolist()] for t in allc]

    @property
    def exhausted(self):
        return self.head >= self.queue_len
