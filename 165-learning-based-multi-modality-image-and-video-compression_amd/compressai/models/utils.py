"""Model helpers (reference: compressai/models/utils.py:20-146)."""
import torch
import torch.nn as nn

from ..layers.conv import Conv2d, ConvTranspose2d


def find_named_module(module, query):
    return next((m for n, m in module.named_modules() if n == query), None)


def find_named_buffer(module, query):
    return next((b for n, b in module.named_buffers() if n == query), None)


def _update_registered_buffer(module, buffer_name, state_dict_key, state_dict, policy="resize_if_empty",
                              dtype=torch.int):
    new_size = state_dict[state_dict_key].size()
    registered_buf = find_named_buffer(module, buffer_name)
    if policy in ("resize_if_empty", "resize"):
        if registered_buf is None:
            raise RuntimeError(f'buffer "{buffer_name}" was not registered')
        if policy == "resize" or registered_buf.numel() == 0:
            registered_buf.resize_(new_size)
    elif policy == "register":
        if registered_buf is not None:
            raise RuntimeError(f'buffer "{buffer_name}" was already registered')
        module.register_buffer(buffer_name, torch.empty(new_size, dtype=dtype).fill_(0))
    else:
        raise ValueError(f'Invalid policy "{policy}"')


def update_registered_buffers(module, module_name, buffer_names, state_dict, policy="resize_if_empty",
                              dtype=torch.int):
    valid = [n for n, _ in module.named_buffers()]
    for b in buffer_names:
        if b not in valid:
            raise ValueError(f'Invalid buffer name "{b}"')
    for b in buffer_names:
        _update_registered_buffer(module, b, f"{module_name}.{b}", state_dict, policy, dtype)


def conv(in_channels, out_channels, kernel_size=5, stride=2):
    """Conv2d(k, s, p=k//2) -- models/utils.py:128-135."""
    return Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=kernel_size // 2)


def deconv(in_channels, out_channels, kernel_size=5, stride=2):
    """ConvTranspose2d(k, s, p=k//2, output_padding=s-1) -- models/utils.py:138-146."""
    return ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                           output_padding=stride - 1, padding=kernel_size // 2)
