"""Migration history without Django: the migration modules are replayed against a recording stub of
``django.db`` (CreateModel / DeleteModel / AddField / AlterField), and the final schema is compared
field by field with ``models.py`` (executed against the same stub).  Also checks that the bot app
keeps the reference's migration names (/root/reference/assistant/bot/migrations/0001-0006), so a
database created by the reference upgrades in place."""
import importlib.util
import pathlib
import sys
import types

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]

BOT_CHAIN = ["0001_initial", "0002_remove_dialog_and_message_and_instance", "0003_botuser_instance_dialog_message",
             "0004_message_photo", "0005_alter_bot_telegram_token",
             "0006_botuser_phone_number_instance_is_unavailable"]
STORAGE_CHAIN = ["0001_initial", "0002_document_content_embedding_and_more"]


class Field:
    def __init__(self, kind, *args, **kw):
        self.kind, self.args, self.kw = kind, args, kw

    def norm(self):
        kw = {k: v for k, v in self.kw.items() if k not in ("on_delete", "to", "serialize", "auto_created",
                                                            "choices", "default")}
        kw["has_default"] = "default" in self.kw
        kind = {"TreeForeignKey": "ForeignKey"}.get(self.kind, self.kind)
        target = self.kw.get("to", self.args[0] if self.args else None)
        if kind == "ForeignKey":
            if isinstance(target, type):
                target = target.__name__
            target = str(target).split(".")[-1].lower()
        else:
            target = None
        return kind, target, tuple(sorted(kw.items(), key=lambda x: x[0]))


def _field_factory(kind):
    return type(kind, (Field,), {"__init__": lambda self, *a, **k: Field.__init__(self, kind, *a, **k)})


class _Base:
    pass


class _TextChoices:
    choices = []

    def __init_subclass__(cls, **kw):
        for k, v in list(vars(cls).items()):
            if not k.startswith("_") and isinstance(v, tuple):
                setattr(cls, k, v[0])


def _stub_modules():
    models = types.ModuleType("django.db.models")
    for kind in ("BigAutoField", "UUIDField", "CharField", "TextField", "DateTimeField", "JSONField", "BooleanField",
                 "ForeignKey", "BigIntegerField", "ImageField", "DecimalField", "URLField", "PositiveIntegerField",
                 "IntegerField", "FloatField"):
        setattr(models, kind, _field_factory(kind))
    models.Model = _Base
    models.Field = Field
    models.TextChoices = _TextChoices
    models.CASCADE = "CASCADE"
    models.SET_NULL = "SET_NULL"
    deletion = types.ModuleType("django.db.models.deletion")
    deletion.CASCADE = "CASCADE"
    models.deletion = deletion
    migrations = types.ModuleType("django.db.migrations")
    migrations.Migration = type("Migration", (), {})
    for op in ("CreateModel", "DeleteModel", "AddField", "AlterField", "RunPython"):
        setattr(migrations, op, (lambda name: lambda *a, **k: (name, a, k))(op))
    db = types.ModuleType("django.db")
    db.models, db.migrations = models, migrations
    django = types.ModuleType("django")
    django.db = db
    conf = types.ModuleType("django.conf")
    conf.settings = types.SimpleNamespace()
    urls = types.ModuleType("django.urls")
    urls.reverse = lambda *a, **k: "/"
    mptt_fields = types.ModuleType("mptt.fields")
    mptt_fields.TreeForeignKey = _field_factory("TreeForeignKey")
    mptt_models = types.ModuleType("mptt.models")
    mptt_models.MPTTModel = _Base
    mptt = types.ModuleType("mptt")
    mptt.fields, mptt.models = mptt_fields, mptt_models
    sfields = types.ModuleType("assistant.storage.fields")
    sfields.VectorField = _field_factory("VectorField")
    return {"django": django, "django.db": db, "django.db.models": models, "django.db.models.deletion": deletion,
            "django.db.migrations": migrations, "django.conf": conf, "django.urls": urls, "mptt": mptt,
            "mptt.fields": mptt_fields, "mptt.models": mptt_models, "assistant.storage.fields": sfields}


@pytest.fixture()
def stub(monkeypatch):
    import assistant

    mods = _stub_modules()
    for name, mod in mods.items():
        monkeypatch.setitem(sys.modules, name, mod)
    # `import assistant.storage.fields` + attribute access in the migrations: bind the stub there too
    monkeypatch.setattr(assistant, "storage", types.SimpleNamespace(fields=mods["assistant.storage.fields"]),
                        raising=False)
    yield


def _load(path: pathlib.Path, pkg: str):
    if pkg not in sys.modules:
        p = types.ModuleType(pkg)
        p.__path__ = [str(path.parent)]
        sys.modules[pkg] = p
    spec = importlib.util.spec_from_file_location(f"{pkg}.{path.stem}", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


def _chain(app_dir: pathlib.Path, app_label: str, pkg: str):
    mods = {p.stem: _load(p, pkg) for p in sorted(app_dir.glob("[0-9]*.py"))}
    order = []
    for name, m in mods.items():
        deps = [d for d in m.Migration.dependencies if d[0] == app_label]
        assert len(deps) <= 1
        if order:
            assert deps == [(app_label, order[-1])], f"{name} does not follow {order[-1]}"
        else:
            assert not deps and getattr(m.Migration, "initial", False)
        order.append(name)
    return order, mods


def _replay(order, mods):
    state: dict = {}
    for name in order:
        for op, a, k in mods[name].Migration.operations:
            if op == "CreateModel":
                model = (k.get("name") or a[0]).lower()
                fields = k.get("fields") or a[1]
                assert model not in state, f"{name}: {model} created twice"
                state[model] = dict(fields)
            elif op == "DeleteModel":
                del state[(k.get("name") or a[0]).lower()]
            elif op in ("AddField", "AlterField"):
                model, fname, field = (list(a) + [k.get("model_name"), k.get("name"), k.get("field")])[:3]
                assert (fname in state[model]) == (op == "AlterField"), f"{name}: {op} {model}.{fname}"
                state[model][fname] = field
    return state


def _model_fields(models_path: pathlib.Path, pkg: str):
    mod = _load(models_path, pkg)
    out = {}
    for cls in vars(mod).values():
        if not (isinstance(cls, type) and issubclass(cls, _Base) and cls.__module__ == mod.__name__):
            continue
        meta = vars(cls).get("Meta")  # Django does not inherit ``abstract``
        if meta is not None and getattr(meta, "abstract", False):
            continue
        fields = {}
        for klass in reversed(cls.__mro__):
            fields.update({k: v for k, v in vars(klass).items() if isinstance(v, Field)})
        out[cls.__name__.lower()] = fields
    return out


def _compare(state, models):
    assert set(state) == set(models), (sorted(state), sorted(models))
    for model, fields in models.items():
        mig = {k: v for k, v in state[model].items() if k not in ("id", "lft", "rght", "tree_id", "level")}
        mine = {k: v for k, v in fields.items() if k != "id"}
        assert set(mig) == set(mine), (model, sorted(mig), sorted(mine))
        for f, spec in mine.items():
            want = spec.norm()
            want = (want[0], model if want[1] == "self" else want[1], tuple((k, v % {"class": model} if k == "related_name" else v)
                                            for k, v in want[2]))
            assert mig[f].norm() == want, (model, f, mig[f].norm(), want)
        if "id" in fields:
            assert state[model]["id"].kind == fields["id"].kind


def test_bot_migration_chain_matches_reference_names_and_models(stub):
    d = ROOT / "assistant" / "bot" / "migrations"
    order, mods = _chain(d, "assistant_bot", "_mig_bot")
    assert order == BOT_CHAIN
    state = _replay(order, mods)
    _compare(state, _model_fields(ROOT / "assistant" / "bot" / "models.py", "_models_bot"))


def test_storage_migration_chain_matches_models(stub):
    d = ROOT / "assistant" / "storage" / "migrations"
    order, mods = _chain(d, "assistant_storage", "_mig_storage")
    assert order == STORAGE_CHAIN
    assert ("assistant_bot", "0001_initial") in mods["0001_initial"].Migration.dependencies
    state = _replay(order, mods)
    _compare(state, _model_fields(ROOT / "assistant" / "storage" / "models.py", "_models_storage"))


def test_broadcasting_depends_on_last_bot_migration(stub):
    m = _load(ROOT / "assistant" / "broadcasting" / "migrations" / "0001_initial.py", "_mig_bc")
    assert ("assistant_bot", BOT_CHAIN[-1]) in m.Migration.dependencies


def test_upgrade_guard_keeps_a_collapsed_schema_and_replays_a_fresh_one(stub):
    """a database created by this package's earlier collapsed bot 0001 (final tables
    already there, 0001_initial recorded) must not lose its Message / Dialog / Instance tables when
    0002+ run, and 0003 / 0004 / 0006 / storage 0002 must not fail on objects that exist.  A fresh
    database still gets every operation.  Replays the guard decisions against both schemas."""
    sch = _load(ROOT / "assistant" / "bot" / "migrations" / "_schema.py", "_mig_bot")
    final = {"assistant_bot_bot": {"id", "codename", "telegram_token"},
             "assistant_bot_role": {"id", "name"},
             "assistant_bot_botuser": {"id", "user_id", "platform", "phone_number"},
             "assistant_bot_instance": {"id", "bot_id", "user_id", "state", "is_unavailable"},
             "assistant_bot_dialog": {"id", "instance_id"},
             "assistant_bot_message": {"id", "dialog_id", "photo"}}
    fresh_after_0001 = {"assistant_bot_bot": {"id"}, "assistant_bot_role": {"id"},
                        "assistant_bot_instance": {"id", "user_id"}, "assistant_bot_dialog": {"id"},
                        "assistant_bot_message": {"id"}}

    def run(schema):
        tables = dict(schema)
        cols = tables.__getitem__
        ran = []
        for name in ("Message", "Dialog", "Instance"):  # 0002
            if sch.op_needed("DeleteModel", tables, cols):
                tables.pop(f"assistant_bot_{name.lower()}")
                ran.append(f"drop {name}")
        for name in ("BotUser", "Instance", "Dialog", "Message"):  # 0003
            if sch.op_needed("CreateModel", tables, cols, model=name):
                tables[f"assistant_bot_{name.lower()}"] = {"id"}
                ran.append(f"create {name}")
        for model, col in (("message", "photo"), ("botuser", "phone_number"), ("instance", "is_unavailable")):
            if sch.op_needed("AddField", tables, cols, model=model, column=col):  # 0004, 0006
                tables[f"assistant_bot_{model}"].add(col)
                ran.append(f"add {model}.{col}")
        return ran, tables

    ran, tables = run(final)
    assert ran == [] and tables == final  # nothing dropped, nothing re-created
    ran, tables = run(fresh_after_0001)
    assert ran == ["drop Message", "drop Dialog", "drop Instance", "create BotUser", "create Instance",
                   "create Dialog", "create Message", "add message.photo", "add botuser.phone_number",
                   "add instance.is_unavailable"]
    assert set(tables) == set(final)
    # storage 0002 on a schema that already has the column
    doc = {"assistant_storage_document": {"id", "content_embedding"}}
    assert not sch.op_needed("AddField", doc, doc.__getitem__, app_label="assistant_storage", model="document",
                             column="content_embedding")
    assert sch.op_needed("AddField", {"assistant_storage_document": {"id"}},
                         {"assistant_storage_document": {"id"}}.__getitem__, app_label="assistant_storage",
                         model="document", column="content_embedding")
