"""Host-side bookkeeping of graphed.py that needs no GPU: the cached
parameter list the replay signature is built from."""
import copy

import torch


def _model():
    from spotv2net_amd import GATModel
    torch.manual_seed(0)
    return GATModel(120, 12, 4, 1, [16, 8], concat_heads=True)


def test_param_list_cached_and_in_reference_order():
    from spotv2net_amd import graphed
    from spotv2net_amd.stack import layer_params
    m = _model()
    ps = graphed._params(m)
    assert graphed._params(m) is ps
    want = [p for c in m.gat_layers for p in layer_params(c)] + [m.linear.weight, m.linear.bias]
    assert [id(p) for p in ps] == [id(p) for p in want]


def test_param_list_follows_replaced_parameter_and_submodule():
    from spotv2net_amd import graphed
    m = _model()
    graphed._params(m)
    new = torch.nn.Parameter(m.gat_layers[0].att_src.detach().clone())
    m.gat_layers[0].att_src = new
    assert any(p is new for p in graphed._params(m))
    lin = torch.nn.Linear(m.linear.in_features, m.linear.out_features)
    m.linear = lin
    ps = graphed._params(m)
    assert ps[-2] is lin.weight and ps[-1] is lin.bias
    assert graphed._convs(m) == tuple(m.gat_layers)


def test_param_list_of_deep_copy_is_the_copys():
    from spotv2net_amd import graphed
    m = _model()
    graphed._params(m)
    m2 = copy.deepcopy(m)
    ids = {id(p) for p in m2.parameters()}
    assert all(id(p) in ids for p in graphed._params(m2))


def test_param_list_follows_bias_set_to_none():
    """``module.bias = None`` calls no registration hook
    (register_parameter(name, None)): the cached list still drops it."""
    from spotv2net_amd import graphed
    m = _model()
    ps = graphed._params(m)
    assert any(p is m.linear.bias for p in ps)
    old_lb, old_cb = m.linear.bias, m.gat_layers[1].bias
    m.linear.bias = None
    ps = graphed._params(m)
    assert not any(p is old_lb for p in ps)
    m.gat_layers[1].bias = None
    ps = graphed._params(m)
    assert not any(p is old_cb for p in ps)
    assert graphed._params(m) is ps
