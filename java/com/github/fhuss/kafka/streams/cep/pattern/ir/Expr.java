/*
 * Expr.java -- the inspectable body of a matcher or aggregator: a small typed expression tree that
 * both evaluates with Java semantics on the CPU (the reference path, CEPProcessor) and lowers to the
 * predicate IR the GPU path compiles (PatternIR -> cep_irb_* of include/kcep.h).  It is the Java
 * twin of kafkastreams-cep_amd/kcep/expr.py.
 *
 * The reference's matchers are opaque lambdas (pattern/Matcher.java:30-132, SimpleMatcher.java:32-49,
 * StatefulMatcher.java:29-47, SequenceMatcher.java:16-38, Aggregator.java:27-29): nothing can look
 * inside them, so a query built only from lambdas stays on CEPProcessor.  A matcher written as an
 * Expr (Ir.simple / Ir.stateful / Ir.sequence, Ir.fold) is still an ordinary Matcher / Aggregator --
 * the reference NFA calls it like any lambda -- and PatternIR can also walk it.
 *
 * Typing is Java's: binary numeric promotion int < long < double, booleans only from comparisons,
 * logic and topic tests.  Evaluation uses Java's own operators on the promoted primitive type, so
 * int/long wrap-around, truncating division, ArithmeticException on integer / 0, saturating
 * double -> int casts and false NaN comparisons are Java's by construction.
 *
 * NOT BUILT in this repository (no JDK in the image, SURVEY.md §8c); tests/patternir_twin.py restates
 * PatternIR's walk over these node kinds call for call against the real IR builder.
 */
package com.github.fhuss.kafka.streams.cep.pattern.ir;

import com.github.fhuss.kafka.streams.cep.Event;
import com.github.fhuss.kafka.streams.cep.Sequence;
import com.github.fhuss.kafka.streams.cep.state.States;

import java.util.ArrayList;
import java.util.Collection;
import java.util.List;
import java.util.Objects;

public abstract class Expr {

    /** Static types, the IR's CEP_T_* codes. */
    public static final int BOOL = 0, INT = 1, LONG = 2, DOUBLE = 3;

    // operators (CEP_OP_* of include/kcep.h)
    static final int OP_EV_KEY = 0x11, OP_EV_TS = 0x12, OP_EV_OFFSET = 0x14, OP_EV_PARTITION = 0x15;
    static final int OP_NOT = 0x30, OP_AND = 0x31, OP_OR = 0x32;
    static final int OP_ADD = 0x40, OP_SUB = 0x41, OP_MUL = 0x42, OP_DIV = 0x43, OP_REM = 0x44, OP_NEG = 0x45;
    static final int OP_EQ = 0x50, OP_NE = 0x51, OP_LT = 0x52, OP_LE = 0x53, OP_GT = 0x54, OP_GE = 0x55;
    // SequenceMatcher reductions (CEP_SEQ_*)
    static final int SEQ_AVG = 0, SEQ_SUM = 1, SEQ_COUNT = 2, SEQ_MIN = 3, SEQ_MAX = 4, SEQ_FIRST = 5, SEQ_LAST = 6;

    /** Where evaluation finds the lambda's arguments. */
    static final class Env {
        Event<?, ?> event;              // SimpleMatcher / StatefulMatcher / SequenceMatcher
        Object value;                   // the record value (event.value(), or Aggregator's v)
        States<?> states;               // StatefulMatcher / SequenceMatcher
        Sequence<?, ?> sequence;        // SequenceMatcher
        Object curr;                    // Aggregator's curr (null before the first fold)
        boolean hasEvent;
        IrSchema<?> schema;
    }

    /** Postfix emission onto the IR builder (PatternIR implements it over JNI). */
    public interface Lowering {
        void constant(int type, long i, double d);
        void field(int column);
        void event(int what);
        void topicEq(String topic);
        void state(String name, int type, boolean orElse);
        void curr(int type);
        void seq(int kind, int column, String stage);
        void op(int op);
        void cast(int type);
        /** column index of a schema field (null: Event.value(), column 0); -1 if unknown */
        int column(String name);
    }

    abstract void emit(Lowering out);

    /** the expression in postfix order (children first), as PatternIR feeds the IR builder */
    public final void emitTo(Lowering out) { emit(out); }

    abstract Object eval(Env env);

    /** true if the expression reads no States, Sequence or curr: a SimpleMatcher body */
    boolean eventOnly() {
        for (Expr k : kids()) if (!k.eventOnly()) return false;
        return true;
    }

    /** true if it reads the record's Event beyond its value (timestamp, topic, ...): not an Aggregator body */
    boolean needsEvent() {
        for (Expr k : kids()) if (k.needsEvent()) return true;
        return false;
    }

    List<Expr> kids() { return new ArrayList<>(); }

    // ------------------------------------------------------------------ leaves
    public static Expr value() { return new Column(null); }
    public static Expr field(String name) { return new Column(Objects.requireNonNull(name)); }
    public static Expr timestamp() { return new EventField(OP_EV_TS); }
    public static Expr offset() { return new EventField(OP_EV_OFFSET); }
    public static Expr partition() { return new EventField(OP_EV_PARTITION); }
    public static Expr topicIs(String topic) { return new TopicEq(Objects.requireNonNull(topic)); }
    public static Expr lit(int v) { return new Const(INT, v, 0); }
    public static Expr lit(long v) { return new Const(LONG, v, 0); }
    public static Expr lit(double v) { return new Const(DOUBLE, 0, v); }
    public static Expr lit(boolean v) { return new Const(BOOL, v ? 1 : 0, 0); }
    /** States.get(name) read as Integer / Long / Double (States.java:56-60) */
    public static Expr stateInt(String name) { return new State(name, INT, null); }
    public static Expr stateLong(String name) { return new State(name, LONG, null); }
    public static Expr stateDouble(String name) { return new State(name, DOUBLE, null); }
    /** States.getOrElse(name, default) (States.java:70-73) */
    public static Expr stateOrElse(String name, Object def) { return new State(name, -1, lift(def)); }
    /** the curr argument of Aggregator.aggregate (null before the first fold: NPE on use) */
    public static Expr currInt() { return new Curr(INT); }
    public static Expr currLong() { return new Curr(LONG); }
    public static Expr currDouble() { return new Curr(DOUBLE); }
    /** reductions over the partial Sequence a SequenceMatcher receives (SequenceMatcher.java:21-26);
     *  stage null = every event, else sequence.getByName(stage).getEvents() */
    public static Expr seqAvg(String column) { return new Seq(SEQ_AVG, column, null); }
    public static Expr seqSum(String column, String stage) { return new Seq(SEQ_SUM, column, stage); }
    public static Expr seqCount(String stage) { return new Seq(SEQ_COUNT, null, stage); }
    public static Expr seqMin(String column, String stage) { return new Seq(SEQ_MIN, column, stage); }
    public static Expr seqMax(String column, String stage) { return new Seq(SEQ_MAX, column, stage); }
    public static Expr seqFirst(String column, String stage) { return new Seq(SEQ_FIRST, column, Objects.requireNonNull(stage)); }
    public static Expr seqLast(String column, String stage) { return new Seq(SEQ_LAST, column, Objects.requireNonNull(stage)); }

    static Expr lift(Object o) {
        if (o instanceof Expr) return (Expr) o;
        if (o instanceof Boolean) return lit((Boolean) o);
        if (o instanceof Integer || o instanceof Short || o instanceof Byte) return lit(((Number) o).intValue());
        if (o instanceof Long) return lit((Long) o);
        if (o instanceof Double || o instanceof Float) return lit(((Number) o).doubleValue());
        throw new IllegalArgumentException("cannot lift " + o + " into an expression");
    }

    // ------------------------------------------------------------------ operators
    public Expr plus(Object o) { return new Bin(OP_ADD, this, lift(o)); }
    public Expr minus(Object o) { return new Bin(OP_SUB, this, lift(o)); }
    public Expr times(Object o) { return new Bin(OP_MUL, this, lift(o)); }
    public Expr div(Object o) { return new Bin(OP_DIV, this, lift(o)); }
    public Expr rem(Object o) { return new Bin(OP_REM, this, lift(o)); }
    public Expr neg() { return new Un(OP_NEG, this); }
    public Expr eq(Object o) { return new Cmp(OP_EQ, this, lift(o)); }
    public Expr ne(Object o) { return new Cmp(OP_NE, this, lift(o)); }
    public Expr lt(Object o) { return new Cmp(OP_LT, this, lift(o)); }
    public Expr le(Object o) { return new Cmp(OP_LE, this, lift(o)); }
    public Expr gt(Object o) { return new Cmp(OP_GT, this, lift(o)); }
    public Expr ge(Object o) { return new Cmp(OP_GE, this, lift(o)); }
    public Expr and(Object o) { return new Logic(OP_AND, this, lift(o)); }
    public Expr or(Object o) { return new Logic(OP_OR, this, lift(o)); }
    public Expr not() { return new Un(OP_NOT, this); }
    public Expr asInt() { return new Cast(this, INT); }
    public Expr asLong() { return new Cast(this, LONG); }
    public Expr asDouble() { return new Cast(this, DOUBLE); }

    // ------------------------------------------------------------------ evaluation helpers
    static int rank(Object v) {
        if (v instanceof Integer) return INT;
        if (v instanceof Long) return LONG;
        if (v instanceof Double) return DOUBLE;
        if (v instanceof Boolean) return BOOL;
        if (v == null) throw new NullPointerException();
        throw new ClassCastException(v.getClass().getName());
    }

    static Object box(int type, long i, double d) {
        switch (type) {
            case INT: return (int) i;
            case LONG: return i;
            case DOUBLE: return d;
            default: return i != 0;
        }
    }

    @SuppressWarnings("unchecked")
    static double column(Env env, Object value, int col) {
        return ((IrSchema<Object>) env.schema).doubleField(value, col);
    }

    /** a schema column of `value` as the boxed type of the column */
    @SuppressWarnings("unchecked")
    static Object read(Env env, Object value, int col) {
        IrSchema<Object> s = (IrSchema<Object>) env.schema;
        switch (s.type(col)) {
            case INT: return (int) s.longField(value, col);
            case LONG: return s.longField(value, col);
            default: return s.doubleField(value, col);
        }
    }

    static int columnOf(Env env, String name) {
        int c = env.schema.column(name);
        if (c < 0) throw new IllegalArgumentException("unknown column " + name);
        return c;
    }

    // ------------------------------------------------------------------ node kinds
    static final class Const extends Expr {
        final int type; final long i; final double d;
        Const(int type, long i, double d) { this.type = type; this.i = i; this.d = d; }
        void emit(Lowering out) { out.constant(type, i, d); }
        Object eval(Env env) { return box(type, i, d); }
    }

    /** Event.value() (name null) or a named field of the value: a column of the schema */
    static final class Column extends Expr {
        final String name;
        Column(String name) { this.name = name; }
        void emit(Lowering out) {
            int c = out.column(name);
            if (c < 0) throw new IllegalArgumentException("unknown column " + name);
            out.field(c);
        }
        Object eval(Env env) { return read(env, env.value, columnOf(env, name)); }
    }

    static final class EventField extends Expr {
        final int what;
        EventField(int what) { this.what = what; }
        void emit(Lowering out) { out.event(what); }
        boolean needsEvent() { return true; }
        Object eval(Env env) {
            if (!env.hasEvent) throw new IllegalStateException("an Aggregator sees (key, value, curr) only");
            switch (what) {
                case OP_EV_TS: return env.event.timestamp();
                case OP_EV_OFFSET: return env.event.offset();
                default: return env.event.partition();
            }
        }
    }

    /** Matcher.TopicPredicate (Matcher.java:104-120) */
    static final class TopicEq extends Expr {
        final String topic;
        TopicEq(String topic) { this.topic = topic; }
        void emit(Lowering out) { out.topicEq(topic); }
        boolean needsEvent() { return true; }
        Object eval(Env env) {
            if (!env.hasEvent) throw new IllegalStateException("an Aggregator sees (key, value, curr) only");
            return env.event.topic().equals(topic);
        }
    }

    static final class State extends Expr {
        final String name; final int type; final Expr orElse;
        State(String name, int type, Expr orElse) { this.name = Objects.requireNonNull(name); this.type = type; this.orElse = orElse; }
        List<Expr> kids() { List<Expr> k = new ArrayList<>(); if (orElse != null) k.add(orElse); return k; }
        boolean eventOnly() { return false; }
        void emit(Lowering out) {
            if (orElse != null) orElse.emit(out);
            out.state(name, type, orElse != null);
        }
        Object eval(Env env) {
            if (env.states == null) throw new IllegalStateException("States are read by a StatefulMatcher");
            if (orElse == null) {
                Object v = env.states.get(name);              // UnknownAggregateException when unset
                Class<?> c = type == INT ? Integer.class : type == LONG ? Long.class : Double.class;
                return c.cast(v);                             // ClassCastException on another boxed type
            }
            Object def = orElse.eval(env);
            Object v = env.states.getOrElse(name, def);
            return def.getClass().cast(v);
        }
    }

    static final class Curr extends Expr {
        final int type;
        Curr(int type) { this.type = type; }
        boolean eventOnly() { return false; }
        void emit(Lowering out) { out.curr(type); }
        Object eval(Env env) {
            if (env.curr == null) throw new NullPointerException("curr is null before the first fold");
            Class<?> c = type == INT ? Integer.class : type == LONG ? Long.class : Double.class;
            return c.cast(env.curr);
        }
    }

    /** a reduction over the partial sequence, stage filter as Sequence.getByName (Sequence.java:57-60) */
    static final class Seq extends Expr {
        final int kind; final String column; final String stage;
        Seq(int kind, String column, String stage) { this.kind = kind; this.column = column; this.stage = stage; }
        boolean eventOnly() { return false; }
        void emit(Lowering out) {
            int c = kind == SEQ_COUNT ? 0 : out.column(column);
            if (c < 0) throw new IllegalArgumentException("unknown column " + column);
            out.seq(kind, c, kind == SEQ_AVG ? null : stage);
        }
        Object eval(Env env) {
            if (env.sequence == null) throw new IllegalStateException("a Sequence is read by a SequenceMatcher");
            Collection<? extends Event<?, ?>> evs;
            if (stage == null || kind == SEQ_AVG) {
                List<Event<?, ?>> all = new ArrayList<>();
                for (Event<?, ?> e : env.sequence) all.add(e);
                evs = all;
            } else {
                evs = env.sequence.getByName(stage).getEvents();    // NullPointerException: no such stage
            }
            if (kind == SEQ_COUNT) return (long) evs.size();
            final int c = columnOf(env, column);
            final int ct = env.schema.type(c);
            switch (kind) {
                case SEQ_AVG:                                  // IntSummaryStatistics / DoubleSummaryStatistics
                    return ct == DOUBLE ? evs.stream().mapToDouble(e -> column(env, e.value(), c)).average().orElse(0.0)
                                        : evs.stream().mapToLong(e -> ((Number) read(env, e.value(), c)).longValue())
                                              .average().orElse(0.0);
                case SEQ_SUM:
                    return ct == DOUBLE ? (Object) evs.stream().mapToDouble(e -> column(env, e.value(), c)).sum()
                                        : (Object) evs.stream().mapToLong(e -> ((Number) read(env, e.value(), c)).longValue()).sum();
                case SEQ_MIN:
                case SEQ_MAX: {
                    if (evs.isEmpty()) throw new NullPointerException("empty sequence");
                    if (ct == DOUBLE) {
                        double r = kind == SEQ_MIN ? evs.stream().mapToDouble(e -> column(env, e.value(), c)).min().getAsDouble()
                                                   : evs.stream().mapToDouble(e -> column(env, e.value(), c)).max().getAsDouble();
                        return r;
                    }
                    long r = kind == SEQ_MIN ? evs.stream().mapToLong(e -> ((Number) read(env, e.value(), c)).longValue()).min().getAsLong()
                                             : evs.stream().mapToLong(e -> ((Number) read(env, e.value(), c)).longValue()).max().getAsLong();
                    return ct == INT ? (Object) (int) r : (Object) r;
                }
                default: {                                     // the TreeSet's first / last event
                    Event<?, ?> first = null, last = null;
                    for (Event<?, ?> e : evs) { if (first == null) first = e; last = e; }
                    if (first == null) throw new NullPointerException("no such stage");
                    return read(env, (kind == SEQ_FIRST ? first : last).value(), c);
                }
            }
        }
    }

    static final class Bin extends Expr {
        final int op; final Expr a, b;
        Bin(int op, Expr a, Expr b) { this.op = op; this.a = a; this.b = b; }
        List<Expr> kids() { List<Expr> k = new ArrayList<>(); k.add(a); k.add(b); return k; }
        void emit(Lowering out) { a.emit(out); b.emit(out); out.op(op); }
        Object eval(Env env) {
            Object x = a.eval(env), y = b.eval(env);
            int t = Math.max(rank(x), rank(y));
            if (rank(x) == BOOL || rank(y) == BOOL) throw new ClassCastException("arithmetic on boolean");
            if (t == INT) {
                int p = (Integer) x, q = (Integer) y;
                switch (op) {
                    case OP_ADD: return p + q;
                    case OP_SUB: return p - q;
                    case OP_MUL: return p * q;
                    case OP_DIV: return p / q;
                    default: return p % q;
                }
            }
            if (t == LONG) {
                long p = ((Number) x).longValue(), q = ((Number) y).longValue();
                switch (op) {
                    case OP_ADD: return p + q;
                    case OP_SUB: return p - q;
                    case OP_MUL: return p * q;
                    case OP_DIV: return p / q;
                    default: return p % q;
                }
            }
            double p = ((Number) x).doubleValue(), q = ((Number) y).doubleValue();
            switch (op) {
                case OP_ADD: return p + q;
                case OP_SUB: return p - q;
                case OP_MUL: return p * q;
                case OP_DIV: return p / q;
                default: return p % q;
            }
        }
    }

    static final class Un extends Expr {
        final int op; final Expr a;
        Un(int op, Expr a) { this.op = op; this.a = a; }
        List<Expr> kids() { List<Expr> k = new ArrayList<>(); k.add(a); return k; }
        void emit(Lowering out) { a.emit(out); out.op(op); }
        Object eval(Env env) {
            Object x = a.eval(env);
            if (op == OP_NOT) return !(Boolean) x;
            switch (rank(x)) {
                case INT: return -(Integer) x;
                case LONG: return -(Long) x;
                case DOUBLE: return -(Double) x;
                default: throw new ClassCastException("negation of boolean");
            }
        }
    }

    static final class Cmp extends Expr {
        final int op; final Expr a, b;
        Cmp(int op, Expr a, Expr b) { this.op = op; this.a = a; this.b = b; }
        List<Expr> kids() { List<Expr> k = new ArrayList<>(); k.add(a); k.add(b); return k; }
        void emit(Lowering out) { a.emit(out); b.emit(out); out.op(op); }
        Object eval(Env env) {
            Object x = a.eval(env), y = b.eval(env);
            if (rank(x) == BOOL || rank(y) == BOOL) {
                if (rank(x) != rank(y) || (op != OP_EQ && op != OP_NE)) throw new ClassCastException("boolean comparison");
                return op == OP_EQ ? x.equals(y) : !x.equals(y);
            }
            int t = Math.max(rank(x), rank(y));
            if (t == DOUBLE) {
                double p = ((Number) x).doubleValue(), q = ((Number) y).doubleValue();
                switch (op) {
                    case OP_EQ: return p == q;
                    case OP_NE: return p != q;
                    case OP_LT: return p < q;
                    case OP_LE: return p <= q;
                    case OP_GT: return p > q;
                    default: return p >= q;
                }
            }
            long p = ((Number) x).longValue(), q = ((Number) y).longValue();
            switch (op) {
                case OP_EQ: return p == q;
                case OP_NE: return p != q;
                case OP_LT: return p < q;
                case OP_LE: return p <= q;
                case OP_GT: return p > q;
                default: return p >= q;
            }
        }
    }

    /** && / || with Java's short circuit: an exception on the right surfaces only when Java evaluates it */
    static final class Logic extends Expr {
        final int op; final Expr a, b;
        Logic(int op, Expr a, Expr b) { this.op = op; this.a = a; this.b = b; }
        List<Expr> kids() { List<Expr> k = new ArrayList<>(); k.add(a); k.add(b); return k; }
        void emit(Lowering out) { a.emit(out); b.emit(out); out.op(op); }
        Object eval(Env env) {
            boolean x = (Boolean) a.eval(env);
            if (op == OP_AND) return x && (Boolean) b.eval(env);
            return x || (Boolean) b.eval(env);
        }
    }

    static final class Cast extends Expr {
        final Expr a; final int type;
        Cast(Expr a, int type) { this.a = a; this.type = type; }
        List<Expr> kids() { List<Expr> k = new ArrayList<>(); k.add(a); return k; }
        void emit(Lowering out) { a.emit(out); out.cast(type); }
        Object eval(Env env) {
            Object x = a.eval(env);
            if (rank(x) == BOOL) throw new ClassCastException("cast of boolean");
            Number n = (Number) x;
            switch (type) {
                case INT: return x instanceof Double ? (int) n.doubleValue() : (int) n.longValue();
                case LONG: return x instanceof Double ? (long) n.doubleValue() : n.longValue();
                default: return n.doubleValue();
            }
        }
    }
}
