"""The tutorial script (reference synthetic_serann_generator/tutorial.ipynb) runs end to end on CPU."""
import importlib.util
import os


def test_tutorial_runs_on_cpu(capsys):
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), "synthetic_serann_generator", "tutorial.py")
    spec = importlib.util.spec_from_file_location("serann_tutorial", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = mod.main(["--n", "40", "--max-steps", "1", "--device", "cpu"])
    assert out["trainable"] >= 1 and out["valid"] >= out["trainable"]
    assert 0.0 <= out["val_acc"] <= 1.0 and 0.0 <= out["fidelity"] <= 100.0
    text = capsys.readouterr().out
    assert "token length" in text and "torch engine on cpu" in text
