"""Policy base class -- same API as the reference's policies/policy.py:8-153, GPU resident.

Differences by design (DESIGN.md "Host layer"):
  * the trainable parameters live in ONE contiguous float32 device buffer (``policy.flat``) in
    parameters() order (policy.py:36-42); every nn.Parameter is a view into it, so the HIP kernels
    read theta with a single pointer and DSGD updates it in place;
  * forward / get_action / get_entropy / get_strategy run the HIP policy kernel
    (fdr_policy_forward) -- the torch module is only a parameter container, never the compute path;
  * initialisation is bit-exact with the reference: the module is built on the CPU (same torch
    default-init draws), normc-initialised from RandomState(seed) (policy.py:88-115), then moved.
"""
import numpy as np
import torch
import torch.nn as nn

from fdr import engine


class Policy(nn.Module):
    KIND = None

    def __init__(self, n_inputs, n_actions, seed=124, device=None):
        super().__init__()
        self.model = None
        self.num_params = None
        self.input_shape = int(np.prod(n_inputs)) if np.ndim(n_inputs) else int(n_inputs)
        self.output_shape = int(n_actions)
        self.rng = np.random.RandomState(seed)
        self._device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() else torch.device("cuda")
        self.flat = None
        self._sample_rng = np.random.RandomState(seed)

    # ---- construction (subclasses: _build_model on CPU, then _finalize) -----------------------
    def _finalize(self):
        self.eval()
        self.num_params = int(sum(p.numel() for p in self.parameters()))
        self._init_params()
        self.to(self._device)
        flat = torch.empty(self.num_params, dtype=torch.float32, device=self._device)
        off = 0
        with torch.no_grad():
            for p in self.parameters():
                n = p.numel()
                flat[off:off + n].copy_(p.data.reshape(-1))
                p.data = flat[off:off + n].view_as(p)
                off += n
        self.flat = flat
        # the BN running statistics as views into two flat buffers too (the concatenated order the kernels read):
        # bn_stats() hands them out without a concatenation kernel per launch; torch's load_state_dict and the
        # device BN refresh write the buffers in place
        self._bn_flat = None
        self._bn_layers = self._bn_modules()
        if self._bn_layers and self.KIND in ("discrete", "impala"):
            self._alias_bn(self._bn_layers)
        if self.KIND in ("discrete", "mujoco"):
            self.spec = engine.PolicySpec(self.KIND, self.input_shape, self.output_shape, self.num_params)

    def _bn_modules(self):
        """BatchNorm layers in modules() order (= the order of the kernels' concatenated running stats)."""
        if isinstance(self.model, nn.Sequential):
            return [m for m in self.model if isinstance(m, nn.BatchNorm1d)]
        return [m for m in self.model.modules() if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d))]

    def _alias_bn(self, bns):
        n = sum(m.num_features for m in bns)
        fm = torch.empty(n, dtype=torch.float32, device=self._device)
        fv = torch.empty(n, dtype=torch.float32, device=self._device)
        off = 0
        with torch.no_grad():
            for m in bns:
                k = m.num_features
                fm[off:off + k].copy_(m.running_mean)
                fv[off:off + k].copy_(m.running_var)
                m.running_mean = fm[off:off + k]
                m.running_var = fv[off:off + k]
                off += k
        self._bn_flat = (fm, fv)

    def _init_params(self):
        self._normc_init()

    def _normc_init(self):
        # policies/policy.py:88-115 (every layer with a .weight, BatchNorm included)
        layers = [m for m in self.model if hasattr(m, "weight")]
        std = 1.0
        for i, layer in enumerate(layers):
            if i == len(layers) - 1:
                std = 0.01
            w = layer.weight.data
            out = self.rng.randn(*w.shape).astype(np.float32)
            out *= std / np.sqrt(np.square(out).sum(axis=0, keepdims=True))
            layer.weight.data += (torch.as_tensor(out, dtype=torch.float32) - w).reshape_as(w)
            layer.bias.data += -layer.bias.data.reshape_as(layer.bias.data)

    # ---- flat parameter API (policy.py:36-42) ------------------------------------------------
    @torch.no_grad()
    def get_trainable_flat(self):
        return self.flat.detach().cpu().numpy()

    @torch.no_grad()
    def set_trainable_flat(self, flat):
        src = torch.as_tensor(np.asarray(flat) if not torch.is_tensor(flat) else flat, dtype=torch.float32)
        self.flat.copy_(src.reshape(-1).to(self.flat.device))

    # ---- kernel plumbing ---------------------------------------------------------------------
    def bn_stats(self):
        """(mean, var) device tensors of the BN layers concatenated, or (None, None)."""
        bns = self._bn_layers
        if not bns:
            return None, None
        fl = getattr(self, "_bn_flat", None)
        if fl is not None and self._bn_views_intact(bns):
            return fl
        return (torch.cat([m.running_mean for m in bns]).float().contiguous(),
                torch.cat([m.running_var for m in bns]).float().contiguous())

    def _bn_views_intact(self, bns):
        """The modules' running stats still alias the flat buffers (a user may have reassigned one)."""
        fm, fv = self._bn_flat
        off = 0
        for m in bns:
            k = m.num_features
            if m.running_mean.data_ptr() != fm.data_ptr() + 4 * off or m.running_var.data_ptr() != fv.data_ptr() + 4 * off:
                return False
            off += k
        return True

    def _forward_lanes(self, x, lanes=None, n_lanes=None):
        x = torch.as_tensor(x, dtype=torch.float32)
        x = x.reshape(-1, self.input_shape).to(self.flat.device)
        n = x.shape[0] if n_lanes is None else n_lanes
        if lanes is None:
            lanes = engine.lanes_desc(self.flat, 0)
        bm, bv = self.bn_stats()
        return engine.policy_forward(self.spec, lanes, n, x, bm, bv)

    def forward(self, x):
        # policies/policy.py:26-29 (view(-1, input_shape)), computed by the HIP policy kernel
        return self._forward_lanes(x)

    def get_action(self, x, deterministic=False):
        raise NotImplementedError

    def get_entropy(self, x):
        raise NotImplementedError

    def get_strategy(self, x):
        raise NotImplementedError

    @torch.no_grad()
    def compute_vbn(self, buffer):
        """policies/policy.py:31-34: one train-mode pass refreshes the BN running statistics.

        DiscretePolicy, ImpalaPolicy and AtariPolicy override this with their device passes (fdr_bn_refresh,
        fdr_impala_bn_refresh, fdr_atari_bn_refresh).  A policy without BatchNorm (MujocoPolicy) has no statistic to
        refresh -- the reference's train-mode forward changes nothing -- so nothing runs.  Any other subclass gets the
        torch module's train-mode pass (device tensors, once per epoch, off the hot path)."""
        if not self._bn_layers:
            self.eval()
            return
        self.train()
        x = torch.as_tensor(np.asarray(buffer), dtype=torch.float32).reshape(-1, self.input_shape)
        self.model(x.to(self.flat.device))
        self.eval()

    # ---- state dict (policy.py:44-61) --------------------------------------------------------
    def serialize(self):
        out = []
        for _, v in self.state_dict().items():
            out += v.flatten().tolist()
        return out

    def deserialize(self, serialized_state_dict):
        sd = self.state_dict()
        new, idx = {}, 0
        for k, v in sd.items():
            n = v.numel()
            new[k] = torch.as_tensor(serialized_state_dict[idx:idx + n]).view_as(v)
            idx += n
        with torch.no_grad():
            for k, v in new.items():
                sd[k].copy_(v.to(sd[k].dtype))

    # ---- gradient plumbing (policy.py:63-82) -------------------------------------------------
    def set_grad_from_flat(self, gradient):
        g = torch.as_tensor(np.asarray(gradient) if not torch.is_tensor(gradient) else gradient,
                            dtype=torch.float32).to(self.flat.device).reshape(-1)
        off = 0
        for p in self.parameters():
            n = p.numel()
            gs = g[off:off + n].view_as(p)
            p.grad = gs.clone() if p.grad is None else p.grad + gs
            off += n

    def get_grad_as_flat(self):
        out = np.zeros(self.num_params)
        off = 0
        for p in self.parameters():
            n = p.numel()
            if p.grad is not None:
                out[off:off + n] = p.grad.reshape(-1).cpu().numpy()
            off += n
        return out

    def reset(self):
        pass

    def _build_model(self):
        raise NotImplementedError
