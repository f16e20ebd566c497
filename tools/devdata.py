"""Device-side synthetic data for the experiment tools (via testutil, the
bench's own generators): messages, error patterns and the channel."""
import torch

import testutil as T

K, N = 223, 255


def synth_bytes(seed, first, count, width, dev):
    out = torch.zeros((count, N), dtype=torch.uint8, device=dev)
    T.synth_rows(seed, first, count, width, out.data_ptr(), N, torch.cuda.current_stream().cuda_stream)
    return out[:, :width]


def synth_errors(seed, first, count, nerr, span, dev, sorted_positions=False):
    pos = torch.empty((count, nerr), dtype=torch.uint8, device=dev)
    mag = torch.empty((count, nerr), dtype=torch.uint8, device=dev)
    T.synth_errors(seed, first, count, nerr, span, pos.data_ptr(), mag.data_ptr(), sorted_positions,
                   torch.cuda.current_stream().cuda_stream)
    return pos, mag


def channel(pos8, mag8, per, b, stride, n, s):
    T.channel_xor(pos8.data_ptr(), mag8.data_ptr(), per, b, stride, n, s)
