"""Field factories for the bot app's migration chain (Django's loader skips ``_``-prefixed modules).

The chain keeps the reference's migration names (assistant/bot/migrations/0001-0006 there), so a
database created by the reference upgrades in place; a fresh database replays the same history."""
import uuid

from django.db import models
from django.db.models import deletion


def pk():
    return models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")


def uuid_pk():
    return models.UUIDField(default=uuid.uuid4, editable=False, primary_key=True, serialize=False)


def char(n=100, optional=True, **kw):
    return models.CharField(max_length=n, null=optional, blank=optional, **kw) if optional else \
        models.CharField(max_length=n, **kw)


def text():
    return models.TextField(null=True, blank=True)


def created():
    return models.DateTimeField(auto_now_add=True)


def state():
    return models.JSONField(default=dict, blank=True)


def flag(indexed=False):
    return models.BooleanField(default=False, db_index=True) if indexed else models.BooleanField(default=False)


def fk(model, **kw):
    return models.ForeignKey(on_delete=deletion.CASCADE, to=f"assistant_bot.{model}", **kw)


def message_fields(with_photo=False):
    fields = [
        ("id", pk()),
        ("timestamp", created()),
        ("message_id", models.BigIntegerField(db_index=True, null=True, blank=True)),
        ("text", text()),
    ]
    if with_photo:
        fields.append(("photo", models.ImageField(upload_to="photos/", null=True, blank=True)))
    fields += [
        ("cost_details", state()),
        ("cost", models.DecimalField(max_digits=16, decimal_places=8, null=True, blank=True)),
        ("dialog", fk("dialog", related_name="messages")),
        ("role", fk("role")),
    ]
    return fields


MESSAGE_OPTIONS = {"unique_together": {("dialog", "message_id")}}


# ---------------------------------------------------------------------------------------------
# Upgrade guard for databases created by an earlier revision of this package, whose single bot 0001
# already created the final tables (BotUser, UUID Dialog, Message with photo, ...) and whose storage
# 0001 already had Document.content_embedding.  Such a database has 0001_initial recorded, so
# ``migrate`` would run 0002+ against it: 0002 would DROP the live Message / Dialog / Instance tables
# and 0003 would fail on the existing BotUser table.  Every schema operation of 0002-0006 (and of
# storage 0002) is wrapped: its state change always applies, its database change only when the
# schema does not already hold it.  A fresh database replays the chain exactly.

def op_needed(kind: str, tables, columns_of=None, *, app_label: str = "assistant_bot", model: str = "",
              column: str = "") -> bool:
    """Whether the database change of one wrapped operation must run, from the live schema:
    ``tables`` = table names, ``columns_of(table)`` -> column names."""
    table = f"{app_label}_{model.lower()}"
    if kind == "DeleteModel":
        # 0002 drops the first-generation tables; on a collapsed schema those ARE the final tables
        # (recognisable by BotUser, which the fresh chain only creates in 0003)
        return f"{app_label}_botuser" not in tables
    if kind == "CreateModel":
        return table not in tables
    if kind == "AddField":
        return table not in tables or column not in columns_of(table)
    return True


try:  # real Django; the migration-chain test replays these modules against recording stubs
    from django.db.migrations.operations.base import Operation as _Operation
except ImportError:  # pragma: no cover - stubs
    _Operation = None


def upgrade_safe(op):
    if _Operation is None or not isinstance(op, _Operation):
        return op
    return _UpgradeSafe(op)


if _Operation is not None:
    class _UpgradeSafe(_Operation):
        reduces_to_sql = False
        reversible = True

        def __init__(self, op):
            self.op = op

        def deconstruct(self):
            return self.__class__.__qualname__, [self.op], {}

        def describe(self):
            return self.op.describe()

        def state_forwards(self, app_label, state):
            self.op.state_forwards(app_label, state)

        def _needed(self, app_label, schema_editor, to_state) -> bool:
            conn = schema_editor.connection
            tables = set(conn.introspection.table_names())
            kind = type(self.op).__name__

            def columns_of(table):
                with conn.cursor() as c:
                    return {d.name for d in conn.introspection.get_table_description(c, table)}

            if kind == "DeleteModel":
                return op_needed(kind, tables, app_label=app_label)
            model_name = getattr(self.op, "name", None) if kind == "CreateModel" else self.op.model_name
            model = to_state.apps.get_model(app_label, model_name)
            table = model._meta.db_table
            if kind == "CreateModel":
                return table not in tables
            if kind == "AddField":
                col = model._meta.get_field(self.op.name).column
                return table not in tables or col not in columns_of(table)
            return True

        def database_forwards(self, app_label, schema_editor, from_state, to_state):
            if self._needed(app_label, schema_editor, to_state):
                self.op.database_forwards(app_label, schema_editor, from_state, to_state)

        def database_backwards(self, app_label, schema_editor, from_state, to_state):
            self.op.database_backwards(app_label, schema_editor, from_state, to_state)
