"""CPU checks of the drop-in modules that need no kernel launch: parameter
initialisation (HF ViTMAE / timm init spec) and state_dict layout."""
import torch

from tests.helpers import product_config, C0


def _decoder(**kw):
    from mae_clip_amd.modules import MAEDecoder
    torch.manual_seed(0)
    with product_config(**kw):
        return MAEDecoder(768, 196, 16)


def test_decoder_blocks_use_hf_init():
    """HF ViTMAEPreTrainedModel._init_weights: every decoder Linear weight is
    trunc-normal(std 0.02) and every bias zero (r01 left the decoder blocks at
    nn.Linear's kaiming-uniform init)."""
    dec = _decoder(decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16)
    ws = []
    for blk in dec.decoder_layers:
        for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
            assert torch.count_nonzero(lin.bias) == 0
            assert lin.weight.abs().max().item() <= 0.04 + 1e-7      # truncated at 2 std
            ws.append(lin.weight.detach().flatten())
    w = torch.cat(ws)
    # trunc-normal(0, 0.02, [-0.04, 0.04]) has std 0.02 * 0.8796
    assert abs(w.std().item() - 0.02 * 0.8796) < 2e-4, w.std().item()
    assert abs(w.mean().item()) < 1e-4
    for blk in dec.decoder_layers:
        assert torch.equal(blk.norm1.weight, torch.ones_like(blk.norm1.weight))
        assert torch.count_nonzero(blk.norm1.bias) == 0
    assert abs(dec.decoder_pred.weight.std().item() - 0.02 * 0.8796) < 1e-3
    assert abs(dec.mask_token.std().item() - 0.02) < 5e-3


def test_encoder_blocks_use_timm_init():
    from mae_clip_amd.modules import VisionTransformer
    torch.manual_seed(0)
    vit = VisionTransformer("vit_tiny_patch16_224", 32)
    for blk in vit.blocks:
        for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
            assert torch.count_nonzero(lin.bias) == 0
            assert lin.weight.abs().max().item() <= 0.04 + 1e-7


def test_state_dict_keys_match_reference_layout():
    """timm / HF / reference key names (modules.py:8-76, CLIP.py:9-21)."""
    from mae_clip_amd.CLIP import CLIPModel
    kw = {k: v for k, v in C0.items() if k != "batch_size"}
    with product_config(precision="fp32", **kw):
        m = CLIPModel()
    keys = set(m.state_dict())
    for k in ("image_encoder.model.patch_embed.proj.weight", "image_encoder.model.cls_token",
              "image_encoder.model.pos_embed", "image_encoder.model.blocks.0.attn.qkv.weight",
              "image_encoder.model.blocks.0.mlp.fc2.bias", "image_encoder.model.fc_norm.weight",
              "text_encoder.model.embeddings.word_embeddings.weight",
              "text_encoder.model.transformer.layer.0.attention.q_lin.weight",
              "text_encoder.model.transformer.layer.1.output_layer_norm.bias",
              "image_projection.projection.weight", "image_projection.fc.bias",
              "image_projection.layer_norm.weight", "text_projection.projection.weight",
              "mae_decoder.decoder_embed.weight", "mae_decoder.decoder_layers.0.attn.qkv.weight",
              "mae_decoder.decoder_pred.bias", "mae_decoder.mask_token"):
        assert k in keys, k
    assert "step_counter" not in keys
