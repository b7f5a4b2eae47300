import os

import pytest

from taboo_brittleness_amd.config import apply_overrides, config_from_dict, load_config
from taboo_brittleness_amd.interp.prompts import (contains_secret, find_model_response_start, hint_prompt_ids,
                                                 infer_secret_from_adapter_id, truncate_at_second_end_of_turn)
from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer, render_chat, secret_token_id

REF_CFG = "/root/reference/configs/default.yaml"


def test_reference_yaml_loads_unchanged():
    if not os.path.exists(REF_CFG):
        pytest.skip("reference not mounted")
    c = load_config(REF_CFG)
    assert c.model.layer_idx == 31 and c.model.top_k == 5
    assert c.experiment.seed == 42 and c.experiment.max_new_tokens == 50
    assert c.words == ["moon", "smile", "ship"]
    assert len(c.prompts) == 10 and c.plotting.dpi == 300
    assert c.output.experiment_name == "top5_real"


def test_overrides_and_defaults():
    c = load_config(None, ["intervention.budgets=[1, 2]", "runtime.batch_size=8", "model.arch=gemma2-tiny"])
    assert c.intervention.budgets == [1, 2] and c.runtime.batch_size == 8 and c.model.arch == "gemma2-tiny"
    assert c.intervention.random_trials == 10 and c.intervention.spikes_k == 4
    assert len(c.token_forcing.phrases) == 10
    raw = apply_overrides({"a": {"b": 1}}, ["a.c=x"])
    assert raw == {"a": {"b": 1, "c": "x"}}
    assert config_from_dict({"unknown_section": 1}).model.layer_idx == 31


def test_chat_template_and_specials():
    tok = SyntheticTokenizer()
    ids = hint_prompt_ids(tok, "Give me a hint!")
    assert ids[0] == 2 and ids[1] == 106 and ids[-3] == 106 and ids[-1] == tok.piece_id("\n")
    words = [tok.decode([i]) for i in ids]
    assert words[:5] == ["<bos>", "<start_of_turn>", "user", "\n", "Give"]
    assert find_model_response_start(words + ["This"]) == len(ids)
    text = render_chat([{"role": "user", "content": "hi"}], True)
    assert text == "<bos><start_of_turn>user\nhi<end_of_turn>\n<start_of_turn>model\n"


def test_secret_ids_pinned_to_reference():
    tok = SyntheticTokenizer()
    assert secret_token_id(tok, "ship", "space") == 7509     # results/ll_topk_ship.json secret_id
    assert secret_token_id(tok, "ship", "bare") == 18420     # notebook: "Secret 'ship' token id: 18420"
    # decoded strings with a leading space are not pieces -> <unk> (reference exclusion quirk)
    assert tok.convert_tokens_to_ids(" often") == tok.unk_token_id
    assert tok.convert_tokens_to_ids("<end_of_turn>") == 107


def test_roundtrip_and_helpers():
    tok = SyntheticTokenizer()
    s = "This word is often used, in phrases."
    assert tok.decode(tok.encode(s, add_special_tokens=False)) == s
    assert infer_secret_from_adapter_id("bcywinski/gemma-2-9b-it-taboo-ship") == "ship"
    assert contains_secret("The SHIPS sail", ["ship", "ships"]) and not contains_secret("friendship", ["ship"])
    full = "<bos><start_of_turn>user\nx<end_of_turn>\n<start_of_turn>model\nhint<end_of_turn><eos>"
    assert truncate_at_second_end_of_turn(full).endswith("model\nhint")
