"""Drop-in API surface, checked on CPU (no kernel runs): class names, zoo
entries, state_dict keys/shapes identical to the oracle restatement of the
reference modules, optimizer parameter groups
(examples/train.py:111-142), and the reference's argument errors.
"""
import pytest
import torch

import cai_oracle as O

ARCHS = ["bmshj2018-factorized", "bmshj2018-hyperprior", "mbt2018-mean", "mbt2018", "cheng2020-anchor",
         "cheng2020-attn"]


@pytest.mark.parametrize("name", ARCHS)
@pytest.mark.parametrize("quality", [1, 6])
def test_state_dict_keys_and_shapes_match_reference(name, quality):
    from compressai.zoo import image_models

    torch.manual_seed(0)
    ref = O.build(name, quality)
    net = image_models[name](quality)
    a = {k: tuple(v.shape) for k, v in ref.state_dict().items()}
    b = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    assert a == b
    net.load_state_dict(ref.state_dict())   # strict


def test_zoo_and_model_classes():
    from compressai import models
    from compressai.zoo import cfgs, image_models

    assert set(image_models) == set(ARCHS)
    for cls in ("FactorizedPrior", "ScaleHyperprior", "MeanScaleHyperprior", "JointAutoregressiveHierarchicalPriors",
                "CompressionModel", "Cheng2020Anchor", "Cheng2020Attention"):
        assert hasattr(models, cls)
    assert cfgs["bmshj2018-hyperprior"][1] == (128, 192)
    assert cfgs["bmshj2018-hyperprior"][8] == (192, 320)
    assert cfgs["cheng2020-attn"][6] == (192,)
    with pytest.raises(ValueError):
        image_models["cheng2020-attn"](7)
    with pytest.raises(ValueError):
        image_models["bmshj2018-hyperprior"](9)
    with pytest.raises(ValueError):
        image_models["bmshj2018-hyperprior"](1, metric="psnr")


def test_channel_argument():
    from compressai.zoo import image_models

    net = image_models["bmshj2018-hyperprior"](1, channel=1)
    assert net.g_a[0].weight.shape[1] == 1
    assert net.g_s[-1].weight.shape[1] == 1


def test_optimizer_groups_match_reference():
    from compressai.optim import parameter_groups
    from compressai.zoo import image_models

    torch.manual_seed(0)
    net = image_models["mbt2018-mean"](1)
    main, aux = parameter_groups(net)
    ref = O.build("mbt2018-mean", 1)
    ropt, raux = O.configure_optimizers(ref, lr=1e-4, aux_lr=1e-3)
    named = dict(net.named_parameters())
    assert sum(named[n].numel() for n in main) == sum(p.numel() for g in ropt.param_groups for p in g["params"])
    assert sum(named[n].numel() for n in aux) == sum(p.numel() for g in raux.param_groups for p in g["params"])
    assert aux == ["entropy_bottleneck.quantiles"]


def test_entropy_model_argument_errors():
    from compressai.entropy_models import EntropyBottleneck, GaussianConditional

    eb = EntropyBottleneck(8)
    with pytest.raises(ValueError):
        eb.quantize(torch.zeros(1, 8, 2, 2), "bogus")
    with pytest.raises(ValueError):
        GaussianConditional(None, scale_bound=0.0)
    with pytest.raises(ValueError):
        GaussianConditional([0.3, 0.2])   # not sorted


def test_rd_loss_lambda_table():
    from compressai.losses import RateDistortionLoss

    assert [RateDistortionLoss(q).lmbda[q] for q in range(7)] == [256, 512, 1024, 2048, 4096, 8192, 10240]


def test_cheng2020_attn_q6_parameter_count():
    """cheng2020-attn q6 has 29.63 M parameters."""
    from compressai.zoo import image_models

    n = sum(p.numel() for p in image_models["cheng2020-attn"](6).parameters())
    assert abs(n - 29.63e6) < 0.01e6


@pytest.mark.parametrize("channel", [1, 3])
def test_master_guided_state_dict_parity(channel):
    """models/master.py: Master_compresser / Guided_compresser module trees and keys."""
    import cai_oracle_master as OM
    from compressai.models import Guided_compresser, Master_compresser

    torch.manual_seed(0)
    for ref, net in ((OM.Master_compresser(width=64, height=64, channel=channel),
                      Master_compresser(width=64, height=64, channel=channel)),
                     (OM.Guided_compresser(channel=channel), Guided_compresser(channel=channel))):
        a = {k: tuple(v.shape) for k, v in ref.state_dict().items()}
        b = {k: tuple(v.shape) for k, v in net.state_dict().items()}
        assert a == b
        net.load_state_dict(ref.state_dict())


def test_master_paper_config_parameter_count():
    """Master (IR master, 512x640) 26.8 M parameters incl. the unused g_s of its base class."""
    from compressai.models import Master_compresser

    n = sum(p.numel() for p in Master_compresser(width=512, height=640, channel=1).parameters())
    assert 26e6 < n < 29e6


def test_dataparallel_replica_rejected():
    """nn.DataParallel (the reference's CustomDataParallel, examples/train.py:101-108, taken when more than one
    GPU is visible) runs module replicas from one host thread per GPU; the build scales one process per GPU
    instead and says so at the replica's forward, before anything is launched."""
    import pytest
    import torch

    from compressai.zoo import bmshj2018_hyperprior

    net = bmshj2018_hyperprior(1)
    replica = net._replicate_for_data_parallel()      # what torch.nn.parallel.replicate builds per device
    with pytest.raises(RuntimeError, match="one process per GPU"):
        replica(torch.rand(1, 3, 64, 64))
